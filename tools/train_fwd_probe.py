"""Times the training forward's point kernel (pnr_render_points, k_point_mlp<3, false, false>)
on the cfg5 shapes (4 objects x 256 rays x 64 coarse / 48 fine samples) with and without the
activation save, and the inference kernel on the same points for comparison.
    python tools/train_fwd_probe.py"""
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from pnr import synth, util  # noqa: E402
from pnr.models import make_model  # noqa: E402
from pnr.train import RenderPoints, mlp_params  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
torch.backends.cudnn.benchmark = True
net = make_model(bench.model_conf()).to(dev)
net.load_state_dict(synth.pixelnerf_state(0), strict=False)
net.mlp_precision = "f16x3"
sb, per, H, W = 4, 256, bench.H, bench.W
src = synth.srn_poses([float(15 * i + 7) for i in range(sb)]).to(dev)
tgt = synth.srn_poses([float(15 * i + 97) for i in range(sb)]).to(dev)
focal = torch.tensor(131.25, device=dev)
g = torch.Generator(device=dev).manual_seed(0)
images = torch.rand(sb, 3, H, W, device=dev, generator=g) * 2 - 1
all_rays = util.gen_rays(tgt, W, H, focal, 0.8, 1.8).reshape(sb, -1, 8)
pix = torch.randint(0, W * H, (sb, per), device=dev, generator=g)
rays = torch.gather(all_rays, 1, pix[..., None].expand(-1, -1, 8)).reshape(-1, 8).contiguous()
with torch.no_grad():
    net.encode(images, src, focal)
lat = net.encoder.latent_cl
for K in (64, 48):
    z = (0.8 + torch.sort(torch.rand(rays.shape[0], K, device=dev, generator=g), -1)[0]).contiguous()
    coarse = K == 64
    mlp = net.mlp_coarse if coarse else net.mlp_fine
    params = mlp_params(mlp)
    for name, grad in (("save", True), ("no save", False)):
        ctx = types.SimpleNamespace(needs_input_grad=(grad,) * 8, save_for_backward=lambda *t: None)
        for _ in range(3):
            RenderPoints.forward(ctx, net, coarse, rays, z, lat, *params)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            RenderPoints.forward(ctx, net, coarse, rays, z, lat, *params)
        e1.record()
        torch.cuda.synchronize()
        print("K=%d %-8s %.3f ms per launch (%d points)" % (K, name, e0.elapsed_time(e1) / 20, z.numel()))
