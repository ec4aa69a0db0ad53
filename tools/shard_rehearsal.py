#!/usr/bin/env python3
"""One rank's share of bench.py's cfg3 headline at --gpus N, timed on ONE GPU.

The 8-GPU SCALE run is the driver's; this rehearses its per-rank work on the 1-GPU box:
rank 0's contiguous shard of the 98,304-ray batch (pnr.dist.shard_range(n, 0, N)), the same
step as bench.py's cfg3 leg (encode + latent projection + render in 50,000-ray chunks +
device->host copy), the same RenderProbe HIP events.  No collective runs (the path has none;
bench.py's ranks only meet at the timing barriers), so N x (rays per rank) / (step time) is
the projected whole-job rate at N ranks, and the per-kernel split shows which fixed costs
stop the scaling.  Usage: python tools/shard_rehearsal.py [N ...]   (default 1 2 4 8)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    worlds = [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = bench._lib.load()
    if hasattr(lib, "pnr_render_set_fused"):
        lib.pnr_render_set_fused(2)
    orig = bench.pdist.shard_range

    class A:
        precision, no_latent_proj, steps, warmup = "f16x3", False, 10, 2
        encoder_eager = os.environ.get("ENCODER_EAGER") == "1"   # A/B of pnr.encoder.InferenceTrunk

    for n in worlds:
        bench.pdist.shard_range = lambda total, rank, world, n=n: orig(total, 0, n)
        probe = bench.RenderProbe(bench.HipEvents())
        _, nmr, elapsed, avg, roof, enc_ms, (s, e) = bench.cfg3_leg(A, dev, 0, 1, probe)
        ms = 1e3 * elapsed / A.steps
        kern = sum(v for k, v in avg.items() if k.startswith(("mlp_", "sample_", "composite_")))
        print(json.dumps({
            "world": n, "encoder": "eager" if A.encoder_eager else "folded trunk graph", "rays_per_rank": e - s, "ms_per_step": round(ms, 3),
            "projected_rays_per_s": round(n * (e - s) / (ms / 1e3), 1),
            "encode_ms": round(enc_ms, 3),
            "render_kernels_ms_per_chunk": {k: round(v, 4) for k, v in avg.items()},
            "launch_ms_fine": roof["launch_ms"], "frac": roof["frac"],
            "render_kernel_ms_sum_per_chunk": round(kern, 3)}), flush=True)
    bench.pdist.shard_range = orig


if __name__ == "__main__":
    main()
