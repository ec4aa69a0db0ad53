#!/usr/bin/env python
"""Is the cfg5 training forward (k_point_mlp with the activation save) slow because of the save or
because of its size?  Times pnr.train.RenderPoints.forward on the cfg5 point counts (SB x 256 rays x
64 coarse / 96 fine samples) with the save (parameters requiring grad) and without it (detached
parameters: no save), HIP events on the launch stream, N repeats each, alternating; and the same
two at 8x the points.  Prints ms and the fp32-equivalent TFLOP/s of each."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from pnr import synth, util  # noqa: E402
from pnr.models import make_model  # noqa: E402
from pnr.train import RenderPoints, mlp_params  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
net = make_model(bench.model_conf()).to(dev)
net.load_state_dict(synth.pixelnerf_state(0), strict=False)
net.mlp_precision = "f16x3"
net.train()
sb, per = 4, 256
images = torch.rand(sb, 3, bench.H, bench.W, device=dev) * 2 - 1
poses = synth.srn_poses([float(15 * i + 7) for i in range(sb)]).to(dev)
focal = torch.tensor(131.25, device=dev)
with torch.no_grad():
    net.encode(images, poses, focal)
lat = net.encoder.latent_cl


def run(K, mult, save):
    B = sb * per * mult
    tgt = synth.srn_poses([float(15 * i + 90) for i in range(sb)]).to(dev)
    rays = util.gen_rays(tgt, bench.W, bench.H, focal, 0.8, 1.8).reshape(sb, -1, 8)[:, :per * mult]
    rays = rays.reshape(B, 8).contiguous()
    z = (torch.linspace(0.8, 1.8, K, device=dev)[None].expand(B, K)).contiguous()
    mlp = net.mlp_coarse if K == 64 else net.mlp_fine
    params = mlp_params(mlp) if save else [p.detach() for p in mlp_params(mlp)]
    net.num_objs = sb
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    RenderPoints.apply(net, K == 64, rays, z, lat, *params)
    a.record()
    for _ in range(5):
        out = RenderPoints.apply(net, K == 64, rays, z, lat, *params)
    b.record()
    torch.cuda.synchronize()
    del out
    ms = a.elapsed_time(b) / 5
    return ms, bench.FLOP_PER_POINT_NS1 * B * K / (ms * 1e-3) / 1e12


for rnd in range(2):
    for mult in (1, 8):
        for K in (64, 96):
            r = {s: run(K, mult, s) for s in (True, False)}
            print("round %d  points %7d (K %d x %d rays)  save %.3f ms %.0f TF   no save %.3f ms %.0f TF" % (
                rnd, sb * per * mult * K, K, sb * per * mult, r[True][0], r[True][1], r[False][0], r[False][1]),
                flush=True)
