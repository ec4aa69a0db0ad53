"""Per-point model outputs of one ray, HIP vs oracle (diagnostic)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pixel-nerf_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

import test_gpu_train as t  # noqa: E402
from oracle import ref_cpu  # noqa: E402
from pnr.models import PixelNeRFNet  # noqa: E402

torch.set_num_threads(8)
DEV = "cuda"
cs = t.case(ns=1, kfd=0, kf=16, seed=11)
sb, n = cs["rays"].shape[:2]
rays = cs["rays"].reshape(-1, 8)
z = ref_cpu.sample_coarse(rays, cs["kc"], cs["streams"][0])
r = 9
pts = (rays[r, :3] + z[r, :, None] * rays[r, 3:6])
dirs = rays[r, 3:6].expand(pts.shape[0], 3)
xyz = torch.zeros(sb, pts.shape[0], 3)
vd = torch.zeros(sb, pts.shape[0], 3)
xyz[1], vd[1] = pts, dirs
xyz[0], vd[0] = pts, dirs
sd = cs["sd"]
scene = ref_cpu.Scene(cs["latent"], cs["poses"][:, None], cs["focal"], cs["width"], cs["height"], cs["c"])
with torch.no_grad():
    ref = ref_cpu.pixelnerf_forward(sd, scene, xyz, True, vd)
    ref64 = ref_cpu.pixelnerf_forward({k: v.double() if v.is_floating_point() else v for k, v in sd.items()},
                                      ref_cpu.Scene(cs["latent"].double(), cs["poses"][:, None].double(),
                                                    cs["focal"], cs["width"], cs["height"], cs["c"]),
                                      xyz.double(), True, vd.double())
net = PixelNeRFNet(t.conf())
net.load_state_dict(sd, strict=False)
net = net.to(DEV).eval()
net.mlp_precision = "fp32"
net.encode_latent(cs["latent"].to(DEV), cs["poses"].to(DEV), cs["focal"].to(DEV), (cs["width"], cs["height"]),
                  c=cs["c"].to(DEV), num_objs=sb)
with torch.no_grad():
    got = net(xyz.to(DEV), coarse=True, viewdirs=vd.to(DEV)).cpu()
for k in range(pts.shape[0]):
    print(k, "ref", ["%.7g" % v for v in ref[1, k].tolist()], "fp64", ["%.7g" % v for v in ref64[1, k].tolist()],
          "hip", ["%.7g" % v for v in got[1, k].tolist()])

# composite backward of this ray: torch autograd of the oracle composite vs the HIP kernel
from pnr.train import Composite  # noqa: E402

raw = ref[1].clone().reshape(1, -1, 4).requires_grad_(True)
zr = z[r:r + 1].clone()
ray = rays[r:r + 1].clone()
tgt = cs["target"].reshape(-1, 3)[r:r + 1]
w, rgb, depth = ref_cpu.composite(ray, zr, raw, True)
((rgb - tgt) ** 2).sum().backward()
raw_h = ref[1].clone().reshape(1, -1, 4).to(DEV).requires_grad_(True)
w2, rgb2, depth2 = Composite.apply(zr.to(DEV), raw_h, ray.to(DEV), True)
((rgb2 - tgt.to(DEV)) ** 2).sum().backward()
print("rgb", rgb.tolist(), rgb2.tolist())
for k in range(raw.shape[1]):
    a, b = raw.grad[0, k].tolist(), raw_h.grad[0, k].cpu().tolist()
    if max(abs(x) for x in a + b) > 0:
        print("d_raw", k, ["%.7g" % x for x in a], ["%.7g" % x for x in b])
