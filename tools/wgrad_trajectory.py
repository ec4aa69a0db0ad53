#!/usr/bin/env python
"""Training trajectory under each weight-gradient arithmetic.

The cfg5 training step (bench.py train_leg: SB = 4 objects x 256 rays, 64 coarse + 32 fine (16
depth), encoder + render + MSE(coarse) + MSE(fine) + backward + Adam lr 1e-4; train.py:182-283) on
one fixed synthetic batch per step -- the same rays, targets and injected random streams in every
run, so the runs differ only in their arithmetic:

  fp32       fp32 MFMA forward, fp32 per-layer GEMM backward (pnr/train.py mlp_backward): the baseline
  f16x3      f16x3 forward, fused f16x3 input-gradient chain, f16x3 weight gradients (the default)
  bf16x6     f16x3 forward and chain, bf16x6 weight gradients (net.wgrad_arith = "bf16x6")

For each run: the loss at every step, and after N steps each parameter tensor's distance to the
baseline's, max |p - p_fp32|, relative to how far the baseline moved it, max |p_fp32 - p_0| (a
trajectory that follows the baseline stays far below 1).  ``fp32_repeat`` reruns the baseline: the
training step is not bitwise repeatable (the latent gradient's atomics, MIOpen's convolution
solvers), so its distance is the noise floor the other runs are read against.  Writes one JSON
object to stdout.

  python tools/wgrad_trajectory.py --steps 200
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))

import torch  # noqa: E402

from pnr import synth, util  # noqa: E402
from pnr.models import make_model  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402

RUNS = {"fp32": ("fp32", "f16x3"), "fp32_repeat": ("fp32", "f16x3"), "f16x3": ("f16x3", "f16x3"),
        "bf16x6": ("f16x3", "bf16x6")}


def model_conf():
    mlp = dict(type="resnet", n_blocks=5, d_hidden=512, combine_layer=3, combine_type="average")
    return dict(use_encoder=True, use_xyz=True, use_code=True,
                code=dict(num_freqs=6, freq_factor=1.5, include_input=True), use_viewdirs=True,
                use_code_viewdirs=False, mlp_coarse=mlp, mlp_fine=dict(mlp),
                encoder=dict(backbone="resnet34", pretrained=False, num_layers=4))


def batch(step, dev, sb=4, per=256, W=128, H=128):
    """Step `step`'s synthetic batch: source images / poses, rays, targets, streams (fixed seeds)."""
    g = torch.Generator().manual_seed(1000 + step)
    src = synth.srn_poses([float(37 * step % 360 + 15 * i) for i in range(sb)]).to(dev)
    tgt = synth.srn_poses([float(37 * step % 360 + 15 * i + 90) for i in range(sb)]).to(dev)
    images = (torch.rand(sb, 3, H, W, generator=g) * 2 - 1).to(dev)
    focal = torch.tensor(131.25, device=dev)
    all_rays = util.gen_rays(tgt, W, H, focal, 0.8, 1.8).reshape(sb, -1, 8)
    pix = torch.randint(0, W * H, (sb, per), generator=g).to(dev)
    rays = torch.gather(all_rays, 1, pix[..., None].expand(-1, -1, 8)).contiguous()
    target = torch.rand(sb, per, 3, generator=g).to(dev)
    streams = synth.rng_streams(2000 + step, sb * per, 64, 32, 16)
    return images, src, focal, rays, target, tuple(s.to(dev) for s in streams)


def run(name, steps, dev, batches):
    precision, wgrad = RUNS[name]
    torch.manual_seed(0)   # the same random-init encoder in every run
    net = make_model(model_conf()).to(dev)
    net.load_state_dict(synth.pixelnerf_state(0), strict=False)
    net.mlp_precision = precision
    net.wgrad_arith = wgrad
    net.train()
    p0 = {k: v.detach().clone() for k, v in net.named_parameters()}
    r = NeRFRenderer(n_coarse=64, n_fine=32, n_fine_depth=16, depth_std=0.01, white_bkgd=True).to(dev)
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    mse = torch.nn.functional.mse_loss
    losses = []
    t0 = time.perf_counter()
    for s in range(steps):
        images, src, focal, rays, target, streams = batches[s]
        opt.zero_grad(set_to_none=True)
        net.encode(images, src, focal)
        r.streams = streams
        out = r(net, rays, want_weights=True)
        loss = mse(out.coarse.rgb, target) + mse(out.fine.rgb, target)
        loss.backward()
        opt.step()
        losses.append(float(loss.item()))
    torch.cuda.synchronize(dev)
    return losses, {k: v.detach().clone() for k, v in net.named_parameters()}, p0, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--runs", default="fp32,fp32_repeat,f16x3,bf16x6")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True
    batches = [batch(s, dev) for s in range(args.steps)]
    res = {}
    for name in args.runs.split(","):
        res[name] = run(name, args.steps, dev, batches)
        print("run %s: %.1f s, loss %.6f -> %.6f" % (name, res[name][3], res[name][0][0], res[name][0][-1]),
              file=sys.stderr, flush=True)
    base_l, base_p, p0, _ = res["fp32"]
    out = {"steps": args.steps, "config": "cfg5: SB=4 x 256 rays, 64 + 32 (16 depth), Adam lr 1e-4, encoder trained",
           "runs": {}}
    for name, (losses, params, _, secs) in res.items():
        worst, per = 0.0, {}
        mlp_worst, enc_worst = 0.0, 0.0
        for k, v in params.items():
            moved = float((base_p[k] - p0[k]).abs().max())
            d = float((v - base_p[k]).abs().max())
            rel = d / moved if moved > 0 else (0.0 if d == 0 else float("inf"))
            per[k] = rel
            worst = max(worst, rel)
            if k.startswith("mlp_"):
                mlp_worst = max(mlp_worst, rel)
            elif k.startswith("encoder"):
                enc_worst = max(enc_worst, rel)
        top = sorted(per.items(), key=lambda kv: -kv[1])[:5]
        out["runs"][name] = {
            "arithmetic": {"forward": RUNS[name][0], "weight_grad": RUNS[name][1] if RUNS[name][0] == "f16x3" else
                           "fp32 GEMM"},
            "loss_first": losses[0], "loss_last": losses[-1],
            "loss_every_10": losses[::10],
            "loss_max_rel_dev_vs_fp32": max(abs(a - b) / abs(b) for a, b in zip(losses, base_l)),
            "param_dist_over_fp32_update_max": worst, "mlp_max": mlp_worst, "encoder_max": enc_worst,
            "worst_params": top, "seconds": secs}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
