"""Which ray's loss term carries the HIP-vs-oracle gradient gap (diagnostic)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pixel-nerf_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

import test_gpu_train as t  # noqa: E402
from oracle import ref_cpu  # noqa: E402
from pnr.models import PixelNeRFNet  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402

torch.set_num_threads(8)
DEV = "cuda"
cs = t.case(ns=1, kfd=0, kf=16, seed=11)
sb, n = cs["rays"].shape[:2]


def to64(x):
    if isinstance(x, torch.Tensor) and x.is_floating_point():
        return x.double()
    if isinstance(x, dict):
        return {k: to64(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(to64(v) for v in x)
    return x


def oracle(mask, cs=cs):
    sd = dict(cs["sd"])
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items() if k.startswith("mlp_")}
    sd.update(params)
    latent = cs["latent"].clone().requires_grad_(True)
    scene = ref_cpu.Scene(latent, cs["poses"][:, None], cs["focal"], cs["width"], cs["height"], cs["c"])
    out = ref_cpu.render(lambda p, c, d: ref_cpu.pixelnerf_forward(sd, scene, p, c, d), cs["rays"], cs["kc"],
                         cs["kf"], cs["kfd"], cs["streams"], True, depth_std=0.05)
    loss = (((out["coarse"]["rgb"] - cs["target"]) ** 2).sum(-1) * mask).sum()
    loss.backward()
    return {k: p.grad for k, p in params.items()}


def hip(mask):
    net = PixelNeRFNet(t.conf())
    net.load_state_dict(cs["sd"], strict=False)
    net = net.to(DEV)
    net.mlp_precision = "fp32"
    latent = cs["latent"].to(DEV).requires_grad_(True)
    net.encode_latent(latent, cs["poses"].to(DEV), cs["focal"].to(DEV), (cs["width"], cs["height"]),
                      c=cs["c"].to(DEV), num_objs=sb)
    r = NeRFRenderer(n_coarse=cs["kc"], n_fine=cs["kf"], n_fine_depth=cs["kfd"], depth_std=0.05,
                     white_bkgd=True).to(DEV)
    r.streams = cs["streams"]
    out = r(net, cs["rays"].to(DEV), want_weights=True)
    loss = (((out.coarse.rgb - cs["target"].to(DEV)) ** 2).sum(-1) * mask.to(DEV)).sum()
    loss.backward()
    return {k: p.grad.detach().cpu() for k, p in net.named_parameters() if k.startswith("mlp_coarse")
            and p.grad is not None}


import pnr.train as ptr  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from pnr.train import _save_views  # noqa: E402

_orig = ptr.mlp_backward
REC = []


def rec(mlp, save, d_o, P, ns=1):
    res = _orig(mlp, save, d_o, P, ns)
    REC.append((mlp, d_o.detach().cpu().clone(), P, save.detach().cpu().clone(), res))
    return res


ptr.mlp_backward = rec
mask = torch.zeros(sb * n)
mask[9] = 1.0
hip(mask.reshape(sb, n))
# oracle gradient of ray 9's coarse loss with the model output detached except at rows 315, 316
def oracle_rows(mask, keep):
    sd = dict(cs["sd"])
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items() if k.startswith("mlp_")}
    sd.update(params)
    scene = ref_cpu.Scene(cs["latent"], cs["poses"][:, None], cs["focal"], cs["width"], cs["height"], cs["c"])

    def fn(p, c, d):
        out = ref_cpu.pixelnerf_forward(sd, scene, p, c, d)
        if not c:
            return out
        flat = out.reshape(-1, 4)
        m = torch.zeros(flat.shape[0], 1)
        m[keep] = 1.0
        return (flat * m + flat.detach() * (1 - m)).reshape(out.shape)

    out = ref_cpu.render(fn, cs["rays"], cs["kc"], cs["kf"], cs["kfd"], cs["streams"], True, depth_std=0.05)
    loss = (((out["coarse"]["rgb"] - cs["target"]) ** 2).sum(-1) * mask).sum()
    loss.backward()
    return {k: p.grad for k, p in params.items() if p.grad is not None}


m9 = mask.reshape(sb, n)
full = oracle(m9)
rows = oracle_rows(m9, [315, 316])
others = oracle_rows(m9, [i for i in range(512) if i not in (315, 316)])
REC.clear()
got = hip(m9)
g = REC[0][4][0]
name = {p: k for k, p in REC[0][0].named_parameters()}
gd = {"mlp_coarse." + name[p]: v.detach().cpu() for p, v in g.items()}
for k in ["mlp_coarse.lin_z.2.bias", "mlp_coarse.blocks.1.fc_1.bias"]:
    sc = float(full[k].abs().max())
    print(k, "mlp_backward-rows %.3g" % (float((gd[k] - rows[k]).abs().max()) / sc),
          "final-mlp_backward %.3g" % (float((got[k] - gd[k]).abs().max()) / sc))
for k in ["mlp_coarse.lin_z.2.bias", "mlp_coarse.blocks.1.fc_1.bias", "mlp_coarse.blocks.2.fc_1.bias"]:
    sc = float(full[k].abs().max())
    print(k, "full-rows %.3g" % (float((full[k] - rows[k]).abs().max()) / sc),
          "hip-rows %.3g" % (float((got[k] - rows[k]).abs().max()) / sc),
          "others %.3g" % (float(others[k].abs().max()) / sc if k in others else 0.0))

# pre-activations of rows 315, 316 recomputed in fp64 from the training save: smallest |pre|
mlp, d_o, P, save, res = REC[0]
feat, zl, slot = _save_views(save.double(), P, 5)
sdd = {k: v.double() for k, v in cs["sd"].items() if k.startswith("mlp_coarse")}


def lin(name, x):
    return F.linear(x, sdd["mlp_coarse." + name + ".weight"], sdd["mlp_coarse." + name + ".bias"])


rr = [315, 316]
x = lin("lin_in", feat[rr, :42])
for b in range(5):
    if b < 3:
        x = x + lin("lin_z.%d" % b, zl[rr])
    h = lin("blocks.%d.fc_0" % b, torch.relu(x))
    for nm, pre, sv in [("x%d" % b, x, slot(b)[rr]), ("h%d" % b, h, slot(5 + b)[rr])]:
        a = pre.abs()
        j = int(a.argmin())
        print(nm, "min|pre| %.3g" % float(a.min()), "at", divmod(j, 512), "saved", float(sv.reshape(-1)[j]),
              "flips", int(((pre > 0) != (sv > 0)).sum()))
    x = x + lin("blocks.%d.fc_1" % b, torch.relu(h))
