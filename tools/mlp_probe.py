#!/usr/bin/env python
"""Small driver for counter collection: renders N cfg2 chunks (4096 rays x (64+64))."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402

prec = os.environ.get("PREC", "f16x3")
n = int(os.environ.get("N_CHUNKS", "2"))
dev = torch.device("cuda:0")
sd, net, rays = bench.build_scene(dev, 0)
net.mlp_precision = prec
net.use_latent_proj = os.environ.get("LATENT_PROJ", "1") == "1"
r = NeRFRenderer(n_coarse=64, n_fine=64, white_bkgd=True)
import time  # noqa: E402

import ctypes  # noqa: E402
from pnr import _lib  # noqa: E402

dbg = getattr(_lib.load(), "pnr_debug_phase", None)   # PNR_PHASE_TIMING variant only
ph = (ctypes.c_ulonglong * 16)()
with torch.no_grad():
    r(net, rays[:4096][None])
    torch.cuda.synchronize()
    if dbg is not None:
        dbg(ph, 1)
    t0 = time.perf_counter()
    for i in range(n):
        r(net, rays[:4096][None])
    torch.cuda.synchronize()
print("done", prec, "proj" if net.use_latent_proj else "gather", n, "chunk_ms %.3f" % ((time.perf_counter() - t0) / n * 1e3),
      os.environ.get("PNR_LIB_PATH", "default"))
if dbg is not None:
    dbg(ph, 0)
    v = list(ph)
    sub = ["ray/z loads", "cam loads + transform", "barrier A", "PE + split", "projection", "barrier B"]
    subd = {nm: round(v[k] / max(v[6], 1)) for nm, k in zip(sub, [8, 9, 10, 11, 12, 0])}
    v[0] += sum(v[8:13])   # the features phase is stamped in parts (slots 8-12 + 0)
    names = ["features", "gather", "gemm", "glue", "head"]
    tot = sum(v[:5])
    print("phase cycles/tile (wave 0):", {nm: round(v[i] / v[6]) for i, nm in enumerate(names)},
          "share:", {nm: round(v[i] / tot, 4) for i, nm in enumerate(names)},
          "gemm cycles/call: %.0f" % (v[2] / v[5]), "calls", v[5], "tiles", v[6])
    print("features split (cycles/tile):", subd)

if os.environ.get("COMPOSITE"):
    with torch.no_grad():
        c = bench.composite_roofline(dev, bench.HipEvents())
    print("composite", {k: (v["ms"], v["frac"]) for k, v in c.items()})
