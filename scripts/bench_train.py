#!/usr/bin/env python
"""Training-step benchmark alone (BASELINE.json configs[4]): the `train`
leg of bench.py (bench.train_leg) with its knobs exposed.

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

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from pnr import dist as pdist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sb", type=int, default=4)
    ap.add_argument("--rays-per-obj", type=int, default=256)
    ap.add_argument("--precision", default="f16x3")
    ap.add_argument("--views", type=int, default=1, help="source views per object (train.py -V)")
    ap.add_argument("--bn", choices=["batch", "sync", "frozen"], default=None,
                    help="encoder BatchNorm: batch (per process), sync (over the ranks; default at N > 1), frozen")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step captured as one HIP graph (measured within 1 %% of eager)")
    ap.add_argument("--sync-debug", action="store_true",
                    help="warn on every host-device synchronization inside the timed steps")
    args = ap.parse_args()
    rank, world, local = pdist.init_from_env("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    out = bench.train_leg(dev, rank, world, args.steps, args.warmup, precision=args.precision, sb=args.sb,
                          per=args.rays_per_obj, ns=args.views, graph=args.graph, sync_debug=args.sync_debug)
    out["warmup"] = args.warmup
    out["higher_is_better"] = True
    out["dtype"] = "f32"
    out["data"] = "synthetic (random source images, hash-initialised MLPs, SRN geometry)"
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
