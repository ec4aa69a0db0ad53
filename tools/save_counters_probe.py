#!/usr/bin/env python
"""PMC probe of the training forward's activation save: k_point_mlp<3, false, false> on the cfg5
fine pass (98,304 points, K = 96) 4x WITH the save, then 4x WITHOUT it (detached parameters), in
that order, so a rocprofv3 --pmc run's dispatches of that kernel split into halves
(tools/save_counters.py).  Diagnostic; no output checked."""
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
sb, per, K = 4, 256, 96
images = torch.rand(sb, 3, bench.H, bench.W, device=dev) * 2 - 1
poses = synth.srn_poses([float(15 * i + 7) for i in range(sb)]).to(dev)
focal = torch.tensor(131.25, device=dev)
with torch.no_grad():
    net.encode(images, poses, focal)
tgt = synth.srn_poses([float(15 * i + 90) for i in range(sb)]).to(dev)
rays = util.gen_rays(tgt, bench.W, bench.H, focal, 0.8, 1.8).reshape(sb, -1, 8)[:, :per].reshape(-1, 8).contiguous()
z = torch.linspace(0.8, 1.8, K, device=dev)[None].expand(sb * per, K).contiguous()
net.num_objs = sb
for save in (True, False):
    params = mlp_params(net.mlp_fine) if save else [p.detach() for p in mlp_params(net.mlp_fine)]
    for _ in range(4):
        out = RenderPoints.apply(net, False, rays, z, net.encoder.latent_cl, *params)
    torch.cuda.synchronize()
    del out
print("done")
