"""Activation save of the training forward vs an fp64 re-evaluation from its saved inputs
(diagnostic)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pixel-nerf_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import test_gpu_train as t  # noqa: E402
from oracle import ref_cpu  # noqa: E402
from pnr import _lib  # noqa: E402
from pnr.models import PixelNeRFNet  # noqa: E402
from pnr.train import _save_views  # noqa: E402

DEV = "cuda"
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 11
cs = t.case(ns=1, kfd=0, kf=16, seed=seed)
sb, n = cs["rays"].shape[:2]
rays = cs["rays"].reshape(-1, 8)
z = ref_cpu.sample_coarse(rays, cs["kc"], cs["streams"][0])
net = PixelNeRFNet(t.conf())
net.load_state_dict(cs["sd"], strict=False)
net = net.to(DEV)
net.mlp_precision = "fp32"
net.encode_latent(cs["latent"].to(DEV), cs["poses"].to(DEV), cs["focal"].to(DEV), (cs["width"], cs["height"]),
                  c=cs["c"].to(DEV), num_objs=sb)
mlp = net.mlp_coarse
desc, packed = mlp.packed(net.code, net.mlp_precision)
sc = net.hip_scene()
B, K = z.shape
P = B * K
lib = _lib.load()
save = torch.empty(lib.pnr_point_save_floats(desc, P), dtype=torch.float32, device=DEV)
wsb = lib.pnr_point_query_workspace_bytes(sc, P)
ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=DEV)
out = torch.empty(P, 4, device=DEV)
rd, zd = rays.to(DEV).contiguous(), z.to(DEV).contiguous()
_lib.check(lib.pnr_render_points(sc, desc, _lib.ptr(packed), _lib.Rays(_lib.ptr(rd), B, B // sb), _lib.ptr(zd), K,
                                 _lib.ptr(out), _lib.ptr(save), _lib.ptr(ws), wsb, _lib.stream_of(torch.device(DEV))),
           "render_points")
torch.cuda.synchronize()
save = save.cpu().double()
nb = 5
feat, zl, slot = _save_views(save, P, nb)
sd = {k: v.double() for k, v in cs["sd"].items() if k.startswith("mlp_coarse")}


def lin(name, x):
    return F.linear(x, sd["mlp_coarse." + name + ".weight"], sd["mlp_coarse." + name + ".bias"])


x = lin("lin_in", feat[:, :42])
for b in range(nb):
    if b < 3:
        x = x + lin("lin_z.%d" % b, zl)
    ref_x = torch.relu(x)
    h = lin("blocks.%d.fc_0" % b, ref_x)
    for name, pre, sv in [("x_in %d" % b, x, slot(b)), ("h %d" % b, h, slot(nb + b))]:
        flips = ((pre > 0) != (sv > 0))
        err = (torch.relu(pre) - sv).abs().max().item()
        idx = flips.nonzero()
        print(name, "max|relu - save| %.3g" % err, "flips", int(flips.sum()),
              [(int(i), int(j), "%.3g" % pre[i, j].item(), "%.3g" % sv[i, j].item()) for i, j in idx[:4]])
    x = x + lin("blocks.%d.fc_1" % b, torch.relu(h))
print("out rel err", ((lin("lin_out", torch.relu(x))[:, 3].clamp_min(0) - out.cpu().double()[:, 3]).abs().max()).item())

# mlp_backward on this save vs fp64 autograd of the same network from the saved inputs
from pnr.train import mlp_backward  # noqa: E402

rows = [315, 316]
d_o = torch.zeros(P, 4, dtype=torch.float64)
d_o[rows] = torch.tensor([[0.03, 0.04, 0.004, -0.09], [0.16, 0.23, 0.023, -0.27]], dtype=torch.float64)
g, d_feat, dz = mlp_backward(mlp, save.float().to(DEV), d_o.float().to(DEV), P)
params = {k: v.clone().requires_grad_(True) for k, v in sd.items()}


def lin2(name, x):
    return F.linear(x, params["mlp_coarse." + name + ".weight"], params["mlp_coarse." + name + ".bias"])


x = lin2("lin_in", feat[:, :42])
for b in range(nb):
    if b < 3:
        x = x + lin2("lin_z.%d" % b, zl)
    x = x + lin2("blocks.%d.fc_1" % b, torch.relu(lin2("blocks.%d.fc_0" % b, torch.relu(x))))
o = lin2("lin_out", torch.relu(x))
(o * d_o).sum().backward()
name = {p: k for k, p in mlp.named_parameters()}
for p, gv in g.items():
    k = "mlp_coarse." + name[p]
    ref = params[k].grad
    print("%-36s %.3g" % (k, float((gv.cpu().double() - ref).abs().max()) / max(float(ref.abs().max()), 1e-30)))
