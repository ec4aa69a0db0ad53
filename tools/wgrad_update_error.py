#!/usr/bin/env python
"""Adam-update error of each weight-gradient arithmetic against fp64.

At FIXED parameters (no optimizer step: every sampled step sees the same weights) and fixed
synthetic cfg5 batches (tools/wgrad_trajectory.py batch(): SB = 4 objects x 256 rays, 64 coarse +
32 fine (16 depth); train.py:182-283), each step runs the training forward and the fused f16x3
input-gradient chain once.  Every 512-wide weight gradient G = dY^T X of that backward
(pnr.train.weight_grad: fc_0 / fc_1 of the 5 blocks, the 3 lin_z, coarse and fine MLP) is then
evaluated three ways on the SAME fp32 operands dY and X:

  fp64     torch float64 GEMM (the reference)
  f16x3    k_wgrad_h (the shipped default)
  bf16x6   k_wgrad (split-bf16 products)

so the comparison isolates the weight-gradient arithmetic.  Adam's state (m, v; beta 0.9 / 0.999,
eps 1e-8, torch.optim.Adam's update m_hat / (sqrt(v_hat) + eps)) evolves over the sampled steps on
the fp64 gradients; at every step each arithmetic's gradient is put in place of the fp64 one for
that step's update.  Per (tensor, step): the relative update error ||u - u64|| / ||u64||, the
element-max error max|u - u64| / max|u64|, and the cosine of u with u64.  Reported: max and p99
over all (tensor, step) pairs, and the decision rule of VERDICT r5 item 5 (keep f16x3 if its p99
relative update error is within 2x of bf16x6's).  One JSON object on stdout.

  python tools/wgrad_update_error.py --steps 50
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import torch  # noqa: E402

from pnr import synth  # noqa: E402
from pnr import train as ptrain  # noqa: E402
from pnr.models import make_model  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402
from wgrad_trajectory import batch, model_conf  # noqa: E402

B1, B2, EPS = 0.9, 0.999, 1e-8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = make_model(model_conf()).to(dev)
    net.load_state_dict(synth.pixelnerf_state(0), strict=False)
    net.mlp_precision = "f16x3"
    net.wgrad_arith = "f16x3"
    net.train()
    r = NeRFRenderer(n_coarse=64, n_fine=32, n_fine_depth=16, depth_std=0.01, white_bkgd=True).to(dev)
    mse = torch.nn.functional.mse_loss

    calls = []   # this step's weight_grad operand lists, in call order
    real = ptrain.weight_grad

    def capture(dys, xs, P, arith="f16x3"):
        out = real(dys, xs, P, arith)
        calls.append(([d.clone() for d in dys], [x.clone() for x in xs], P))
        return out

    ptrain.weight_grad = capture
    state = {}   # tensor index -> (m, v) on fp64 gradients
    stats = {"f16x3": [], "bf16x6": []}
    for s in range(args.steps):
        images, src, focal, rays, target, streams = batch(s, dev)
        calls.clear()
        net.zero_grad(set_to_none=True)
        net.encode(images, src, focal)
        r.streams = streams
        out = r(net, rays, want_weights=True)
        loss = mse(out.coarse.rgb, target) + mse(out.fine.rgb, target)
        loss.backward()
        t = s + 1
        idx = 0
        for dys, xs, P in calls:
            g = {"f16x3": real(dys, xs, P, "f16x3"), "bf16x6": real(dys, xs, P, "bf16x6")}
            for j in range(len(dys)):
                g64 = dys[j].double().t() @ xs[j].double()
                m, v = state.get(idx, (torch.zeros_like(g64), torch.zeros_like(g64)))

                def upd(gr):
                    mm = B1 * m + (1 - B1) * gr
                    vv = B2 * v + (1 - B2) * gr * gr
                    return (mm / (1 - B1 ** t)) / ((vv / (1 - B2 ** t)).sqrt() + EPS), mm, vv

                u64, m2, v2 = upd(g64)
                n64 = float(u64.norm())
                for name in stats:
                    u = upd(g[name][j].double())[0]
                    d = u - u64
                    stats[name].append({
                        "tensor": idx, "step": s,
                        "rel": float(d.norm()) / n64 if n64 > 0 else 0.0,
                        "maxrel": float(d.abs().max()) / float(u64.abs().max()) if n64 > 0 else 0.0,
                        "cos": float((u * u64).sum()) / (float(u.norm()) * n64) if n64 > 0 else 1.0,
                        "grad_rel": float((g[name][j].double() - g64).norm()) / max(float(g64.norm()), 1e-300)})
                state[idx] = (m2, v2)
                idx += 1
        print("step %d: %d tensors, loss %.6f" % (s, idx, float(loss)), file=sys.stderr, flush=True)
    ptrain.weight_grad = real

    def q(vals, p):
        vals = sorted(vals)
        return vals[min(len(vals) - 1, int(round(p * (len(vals) - 1))))]

    res = {"steps": args.steps, "tensors_per_step": idx,
           "config": "cfg5 batches (tools/wgrad_trajectory.py), fixed parameters, Adam state on fp64 gradients",
           "arith": {}}
    for name, rows in stats.items():
        res["arith"][name] = {
            "rel_update_err": {"max": max(r_["rel"] for r_ in rows), "p99": q([r_["rel"] for r_ in rows], 0.99),
                               "median": q([r_["rel"] for r_ in rows], 0.5)},
            "elem_max_update_err": {"max": max(r_["maxrel"] for r_ in rows),
                                    "p99": q([r_["maxrel"] for r_ in rows], 0.99)},
            "cos_min": min(r_["cos"] for r_ in rows),
            "grad_rel_err": {"max": max(r_["grad_rel"] for r_ in rows), "p99": q([r_["grad_rel"] for r_ in rows], 0.99)},
            "worst": sorted(rows, key=lambda r_: -r_["rel"])[:3]}
    a, b = res["arith"]["f16x3"]["rel_update_err"]["p99"], res["arith"]["bf16x6"]["rel_update_err"]["p99"]
    res["decision"] = {"rule": "keep f16x3 if its p99 relative update error <= 2 x bf16x6's",
                       "f16x3_p99": a, "bf16x6_p99": b, "ratio": a / b if b > 0 else float("inf"),
                       "keep_f16x3": a <= 2 * b}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
