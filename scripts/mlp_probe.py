#!/usr/bin/env python
"""Small driver for counter collection: renders N cfg2 chunks (4096 rays x (64+64))."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402

prec = os.environ.get("PREC", "bf16x6")
n = int(os.environ.get("N_CHUNKS", "2"))
dev = torch.device("cuda:0")
sd, net, rays = bench.build_scene(dev, 0)
net.mlp_precision = prec
r = NeRFRenderer(n_coarse=64, n_fine=64, white_bkgd=True)
import time  # noqa: E402

with torch.no_grad():
    r(net, rays[:4096][None])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        r(net, rays[:4096][None])
    torch.cuda.synchronize()
print("done", prec, n, "chunk_ms %.3f" % ((time.perf_counter() - t0) / n * 1e3),
      os.environ.get("PNR_LIB_PATH", "default"))
