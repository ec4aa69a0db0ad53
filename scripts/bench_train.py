#!/usr/bin/env python
"""Training-step benchmark (BASELINE.json configs[4]).

One step = the reference's train.py:182-283 on synthetic SRN-cars-shaped data:
  * encode: the ResNet34 trunk (encoder.py:111-164) on SB x NS source images (128x128;
    NS = --views, 1 by default as in the SRN setting, train.py -V);
  * render: SB x B' rays with the shipped conf (64 coarse + 32 fine incl. 16 depth
    samples, white background) through the HIP training path (pnr/train.py);
  * loss: MSE(coarse rgb) + MSE(fine rgb) (lambda = 1, conf/default.conf:77-78);
  * backward;
  * data-parallel gradient mean (bucketed all-reduce, RCCL over xGMI; pnr.dist);
  * Adam (lr 1e-4).

Launch one process per GPU:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
      scripts/bench_train.py --steps K --warmup W
Per-rank work is fixed (weak scaling: SB=4 x 256 rays per rank; 8 ranks = 8192 rays).
Rank 0 prints one JSON line; `value` = rays of all ranks / max-over-ranks step time.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pnr import dist as pdist  # noqa: E402
from pnr import synth, util  # noqa: E402
from pnr.models import make_model  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402


def conf():
    mlp = dict(type="resnet", n_blocks=5, d_hidden=512, combine_layer=3, combine_type="average")
    return dict(use_encoder=True, use_xyz=True, use_code=True,
                code=dict(num_freqs=6, freq_factor=1.5, include_input=True), use_viewdirs=True,
                use_code_viewdirs=False, mlp_coarse=dict(mlp), mlp_fine=dict(mlp),
                encoder=dict(backbone="resnet34", pretrained=False, num_layers=4))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sb", type=int, default=4)
    ap.add_argument("--rays-per-obj", type=int, default=256)
    ap.add_argument("--precision", default="f16x3")
    ap.add_argument("--views", type=int, default=1, help="source views per object (train.py -V)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step captured as one HIP graph instead of launching every kernel "
                         "from Python (measured within 1 %% of eager: the step is GPU-bound)")
    ap.add_argument("--sync-debug", action="store_true",
                    help="warn on every host-device synchronization inside the timed steps")
    args = ap.parse_args()
    rank, world, local = pdist.init_from_env("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    torch.manual_seed(1234 + rank)
    torch.backends.cudnn.benchmark = True   # MIOpen solver search for the encoder convolutions

    net = make_model(conf()).to(dev)
    sd = synth.pixelnerf_state(0)
    net.load_state_dict(sd, strict=False)
    net.mlp_precision = args.precision
    net.train()
    renderer = NeRFRenderer(n_coarse=64, n_fine=32, n_fine_depth=16, depth_std=0.01,
                            white_bkgd=True).to(dev)
    # fused Adam: one multi-tensor kernel per step instead of a host loop of foreach
    # launches (the reference trainer uses torch.optim.Adam, trainer.py:49; same update)
    # capturable: the step counter stays on the device, so the update replays inside a graph
    opt = torch.optim.Adam(net.parameters(), lr=1e-4, fused=True, capturable=args.graph)
    params = list(net.parameters())

    sb, per, ns = args.sb, args.rays_per_obj, args.views
    W = H = 128
    focal = torch.tensor(131.25, device=dev)
    src_poses = synth.srn_poses([float(15 * i + 7 * rank + 40 * v) for i in range(sb) for v in range(ns)]).to(dev)
    if ns > 1:
        src_poses = src_poses.reshape(sb, ns, 4, 4)
    tgt_poses = synth.srn_poses([float(15 * i + 7 * rank + 90) for i in range(sb)]).to(dev)
    g = torch.Generator(device=dev).manual_seed(rank)
    images = torch.rand(sb, 3, H, W, device=dev, generator=g) * 2 - 1 if ns == 1 else \
        torch.rand(sb, ns, 3, H, W, device=dev, generator=g) * 2 - 1
    all_rays = util.gen_rays(tgt_poses, W, H, focal, 0.8, 1.8).reshape(sb, -1, 8)   # on device
    pix = torch.randint(0, W * H, (sb, per), device=dev, generator=g)
    rays = torch.gather(all_rays, 1, pix[..., None].expand(-1, -1, 8)).contiguous()
    target = torch.rand(sb, per, 3, device=dev, generator=g)
    mse = torch.nn.functional.mse_loss

    def step():
        opt.zero_grad(set_to_none=True)
        net.encode(images, src_poses, focal)
        out = renderer(net, rays, want_weights=True)
        loss = mse(out.coarse.rgb, target) + mse(out.fine.rgb, target)
        loss.backward()
        pdist.allreduce_grads(params, world)
        opt.step()
        return loss

    run = step
    if not args.graph:
        for _ in range(args.warmup):
            step()
    else:
        # HIP graph of the whole step (encoder, render, backward, all-reduce, Adam): one replay
        # per step instead of ~540 launches from Python.  Warm-up on a side stream (MIOpen
        # solver search, pack caches, allocator), then capture; inputs are static tensors.
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(max(args.warmup, 2)):
                step()
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(graph):
            static_loss = step()

        def run():
            graph.replay()
            return static_loss

        run()   # first replay
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if args.sync_debug:
        torch.cuda.set_sync_debug_mode("warn")
    for _ in range(args.steps):
        loss = run()
    if args.sync_debug:
        torch.cuda.set_sync_debug_mode("default")
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = pdist.max_over_ranks(time.perf_counter() - t0, dev)
    rays_total = sb * per * args.steps * world
    out = {
        "metric": "training rays/sec (cfg5: encoder + coarse/fine render + backward + grad all-reduce + Adam)",
        "value": round(rays_total / elapsed, 1), "unit": "rays/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "dtype": "f32", "arithmetic": (args.precision + " forward + f16x3 fused input-gradient chain + split-bf16 (x6) weight gradients"
                                                     if args.precision == "f16x3" and ns == 1 else
                                                     args.precision + " forward + fp32 GEMM input-gradient chain + split-bf16 (x6) weight gradients"
                                                     if args.precision == "f16x3" else
                                                     args.precision + " forward, fp32 GEMM backward") + " (pnr/train.py)",
        "data": "synthetic (random source images, hash-initialised MLPs, SRN geometry)",
        "config": {"workload": "cfg5: SB=%d objects x %d rays per rank, %d source view(s), 64 coarse + 32 fine "
                               "(16 depth)" % (sb, per, ns), "global_batch_rays": sb * per * world,
                   "parallelism": "data parallel, 1 process per GPU, bucketed RCCL all-reduce",
                   "launch": "one HIP graph per step" if args.graph else "eager"},
        "loss": round(loss.item(), 6),
    }
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
