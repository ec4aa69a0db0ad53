#!/usr/bin/env python3
"""Diagnostic (GPU): can the next scene's encode hide under the current render?  Rank 0's share of
bench.py's cfg3 step at --gpus N (tools/shard_rehearsal.py's workload), two ways, alternating:
  serial   encode + render on one stream (bench.py's step)
  overlap  two PixelNeRFNets (same weights) used in turn: scene i + 1 is encoded on a side
           stream while scene i renders on the main stream (double-buffered latent, cameras and
           projection); the main stream waits only on the encode of the scene it renders.
k_point_mlp is persistent (one 150 KB-LDS, 512-VGPR-per-SIMD workgroup per CU), so the side
stream's trunk kernels can only take CUs the render leaves free.  Usage: encode_overlap.py [N]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.backends.cudnn.benchmark = True
    nets = [bench.make_net(dev, "f16x3", True, use_first_pool=False) for _ in range(2)]
    img, src, focal, rays = bench.nmr_inputs(dev)
    s, e = bench.pdist.shard_range(rays.shape[0], 0, n)
    mine = rays[s:e]
    rend = NeRFRenderer(n_coarse=bench.KC, n_fine=bench.KF, white_bkgd=True, eval_batch_size=bench.RAY_BATCH).to(dev)
    pars = [rend.bind_parallel(m, simple_output=True).eval() for m in nets]
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    host = torch.empty(e - s, 3, pin_memory=True)

    def render(i):
        outs = [pars[i](r[None])[0][0]
                for r in torch.split(mine, bench.RAY_BATCH, dim=0)]
        host.copy_(torch.cat(outs), non_blocking=True)

    def serial(k):
        for _ in range(k):
            nets[0].encode(img, src, focal)
            render(0)

    def overlap(k):
        evs = [torch.cuda.Event(), torch.cuda.Event()]
        nets[0].encode(img, src, focal)
        evs[0].record(main_s)
        for i in range(k):
            cur, nxt = i % 2, (i + 1) % 2
            if i + 1 < k:
                side.wait_stream(main_s)   # the renders that read nxt's buffers are done
                with torch.cuda.stream(side):
                    nets[nxt].encode(img, src, focal)
                    evs[nxt].record(side)
            main_s.wait_event(evs[cur])
            render(cur)

    with torch.no_grad():
        for f in (serial, overlap):
            f(3)
        torch.cuda.synchronize()
        for rnd in range(3):
            for name, f in (("serial", serial), ("overlap", overlap)):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                f(steps)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / steps * 1e3
                print("N=%d %-8s %.3f ms/step  projected %.1f rays/s" % (n, name, ms, n * (e - s) / ms * 1e3),
                      flush=True)


if __name__ == "__main__":
    main()
