"""Times pnr_mlp_backward_views (k_mlp_bwd) alone on the cfg5 coarse shape (65,536 points, one
view) from a real activation save.  Select a libpnr.so variant with PNR_LIB_PATH.
    python tools/mlp_bwd_probe.py"""
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from pnr import _lib, synth, util  # noqa: E402
from pnr.models import make_model  # noqa: E402
from pnr.train import RenderPoints, mlp_params, _save_views  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
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
K = 64
z = (0.8 + torch.sort(torch.rand(rays.shape[0], K, device=dev, generator=g), -1)[0]).contiguous()
mlp = net.mlp_coarse
saved = {}
ctx = types.SimpleNamespace(needs_input_grad=(True,) * 8, save_for_backward=lambda *t: saved.setdefault("t", t))
RenderPoints.forward(ctx, net, True, rays, z, lat, *mlp_params(mlp))
save = saved["t"][3]
P = z.numel()
desc, packed, packed_t = mlp.packed_t(net.code, net.mlp_precision)
nb = mlp.n_blocks
d_o = torch.randn(P, 4, device=dev, generator=g) * 1e-3
dy = torch.empty(2 * nb + 1, P, 512, device=dev)
dzl = torch.empty(P, 512, device=dev)
w_out = mlp.lin_out.weight.detach().float().contiguous()
sums = torch.empty(2 * nb + 1, 512, device=dev)
lib = _lib.load()
wsb = lib.pnr_mlp_backward_workspace_bytes(desc, P)
ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)


def run():
    _lib.check(lib.pnr_mlp_backward_views(desc, _lib.ptr(packed), _lib.ptr(packed_t), _lib.ptr(w_out), _lib.ptr(save),
                                          _lib.ptr(d_o), P, 1, _lib.ptr(dy), _lib.ptr(dzl), _lib.ptr(sums),
                                          _lib.ptr(ws), wsb, _lib.stream_of(dev)), "pnr_mlp_backward_views")


for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    run()
e1.record()
torch.cuda.synchronize()
print("k_mlp_bwd P=%d: %.3f ms per launch" % (P, e0.elapsed_time(e1) / 20))
