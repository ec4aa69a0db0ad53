#!/usr/bin/env python
"""Diagnostic (GPU): the cfg4 DTU frame (400 x 300 rays, NS = 3 source views, 150 x 200 latent per
view, 64 + 64, gen_video's 50,000-ray chunks; bench.extra_configs' workload) rendered N_FRAMES
times after a warm-up frame, with the library PNR_LIB_PATH selects.  With a PNR_PHASE_TIMING build
it also prints k_point_mlp's phase cycles per tile (as tools/mlp_probe.py)."""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402
from pnr import _lib, synth, util  # noqa: E402
from pnr.models import PixelNeRFNet  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402

n = int(os.environ.get("N_FRAMES", "1"))
dev = torch.device("cuda:0")
sc = synth.scene_multiview(seed=8, n_views=3, n_rays=1)
net = PixelNeRFNet(bench.model_conf())
net.load_state_dict(synth.pixelnerf_state(1), strict=False)
net = net.to(dev).eval()
net.mlp_precision = os.environ.get("PREC", "f16x3")
net.encode_latent(synth.latent(8, 3, 512, 150, 200).to(dev), sc["poses"][None].to(dev), sc["focal"][None].to(dev),
                  (400, 300), c=sc["c"][None].to(dev), num_objs=1)
rays = util.gen_rays(synth.srn_poses([10.0], phi=-12.0, radius=2.0).to(dev), 400, 300, sc["focal"], 0.1, 5.0,
                     c=sc["c"]).reshape(-1, 8)
# ORDER: the frame's ray order -- "row" (gen_rays' row-major, gen_video's), "block:N" (N x N pixel
# blocks, row-major inside and across blocks), "morton" (Z-order of the pixel coordinates), "random"
order = os.environ.get("ORDER", "row")
if order != "row":
    yy, xx = torch.meshgrid(torch.arange(300), torch.arange(400), indexing="ij")
    yy, xx = yy.reshape(-1), xx.reshape(-1)
    if order == "random":
        key = torch.randperm(300 * 400, generator=torch.Generator().manual_seed(0))
    elif order.startswith("block:"):
        nb = int(order.split(":")[1])
        key = ((yy // nb) * ((400 + nb - 1) // nb) + xx // nb) * nb * nb + (yy % nb) * nb + xx % nb
    else:
        key = torch.zeros_like(xx)
        for bit in range(9):
            key |= ((xx >> bit) & 1) << (2 * bit) | ((yy >> bit) & 1) << (2 * bit + 1)
    rays = rays[torch.argsort(key).to(dev)].contiguous()
r = NeRFRenderer(n_coarse=64, n_fine=64, white_bkgd=False,
                 eval_batch_size=int(os.environ.get("EBS", bench.RAY_BATCH))).to(dev)
r.ray_order = os.environ.get("RAY_ORDER", "auto")   # the renderer's processing order (ABI 8)
dbg = getattr(_lib.load(), "pnr_debug_phase", None)
ph = (ctypes.c_ulonglong * 32)()
with torch.no_grad():
    r(net, rays[None])
    torch.cuda.synchronize()
    if dbg is not None:
        dbg(ph, 1)
    t0 = time.perf_counter()
    for _ in range(n):
        r(net, rays[None])
    torch.cuda.synchronize()
print("cfg4 frame_ms %.2f" % ((time.perf_counter() - t0) / n * 1e3), os.environ.get("PNR_LIB_PATH", "default"), order,
      "ray_order=" + r.ray_order, "ebs=%d" % r.eval_batch_size, flush=True)
if dbg is not None:
    dbg(ph, 0)
    v = list(ph)
    v[0] += sum(v[8:13])
    v[3] += sum(v[13:18])
    names = ["features", "gather", "gemm", "glue", "head"]
    tot = sum(v[:5])
    print("phase cycles/tile:", {nm: round(v[i] / max(v[6], 1)) for i, nm in enumerate(names)},
          "share:", {nm: round(v[i] / max(tot, 1), 4) for i, nm in enumerate(names)}, flush=True)
