#!/usr/bin/env python
"""Small driver for counter collection (scripts/counters.sh): renders N_CHUNKS cfg2 chunks
(4096 rays x (64 + 64), SRN geometry, projected latent, precision PREC) after one warm-up
chunk.  With a PNR_PHASE_TIMING build (PNR_LIB_PATH) it also prints the phase counters."""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402
from pnr import _lib, synth, util  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402

prec = os.environ.get("PREC", "f16x3")
n = int(os.environ.get("N_CHUNKS", "2"))
dev = torch.device("cuda:0")
net = bench.make_net(dev, prec, os.environ.get("LATENT_PROJ", "1") == "1")
net.encode_latent(synth.latent(0, 1, 512, 64, 64).to(dev), synth.srn_poses([0.0]).to(dev),
                  torch.tensor(131.25, device=dev), (128, 128))
rays = util.gen_rays(synth.srn_poses([30.0]).to(dev), 128, 128, torch.tensor(131.25), 0.01, 4.0).reshape(-1, 8)
r = NeRFRenderer(n_coarse=64, n_fine=64, white_bkgd=True)
if hasattr(_lib.load(), "pnr_render_set_fused"):
    _lib.load().pnr_render_set_fused(int(os.environ.get("PNR_FUSED", "1")))
dbg = getattr(_lib.load(), "pnr_debug_phase", None)   # PNR_PHASE_TIMING variant only
ph = (ctypes.c_ulonglong * 32)()
with torch.no_grad():
    r(net, rays[:4096][None])
    torch.cuda.synchronize()
    if dbg is not None:
        dbg(ph, 1)
    t0 = time.perf_counter()
    for i in range(n):
        r(net, rays[4096 * (i % 4):4096 * (i % 4 + 1)][None])
    torch.cuda.synchronize()
print("done", prec, "fused", os.environ.get("PNR_FUSED", "1"), n, "chunk_ms %.3f" % ((time.perf_counter() - t0) / n * 1e3), os.environ.get("PNR_LIB_PATH", "default"))
epi = getattr(_lib.load(), "pnr_debug_epi", None)   # PNR_EPI_TIMING variant only
if epi is not None:
    e = (ctypes.c_ulonglong * 8)()
    epi(e)   # since the warm-up (counts include it)
    n_r = max(e[7], 1)
    print("fused epilogue cycles/ray (the epilogue wave):", {nm: round(e[i] / n_r) for i, nm in
          enumerate(["composite", "cdf", "draws", "sort+store"])}, "rays", e[7])
if dbg is not None:
    dbg(ph, 0)
    v = list(ph)
    print("features parts cycles/tile:", {nm: round(v[i] / max(v[6], 1)) for i, nm in
          [(8, "point_loads"), (9, "camera_geometry"), (10, "barrier_in"), (11, "pe_features_split"),
           (12, "projection"), (0, "barrier_out")]})
    v[0] += sum(v[8:13])
    v[3] += sum(v[13:18])   # the publish parts are glue   # the features phase is stamped in parts (slots 8-12 + 0)
    names = ["features", "gather", "gemm", "glue", "head"]
    tot = sum(v[:5])
    extra = {nm: round(v[i] / max(v[6], 1)) for i, nm in [(17, "pre_publish"), (13, "pub_colmax"), (14, "pub_barrier1"),
                                                              (15, "pub_split"), (16, "pub_barrier2")]}
    print("publish parts cycles/tile (wave %s, inside glue):" % os.environ.get("PT_WAVE", "0"), extra)
    print("phase cycles/tile:", {nm: round(v[i] / max(v[6], 1)) for i, nm in enumerate(names)},
          "share:", {nm: round(v[i] / max(tot, 1), 4) for i, nm in enumerate(names)})
