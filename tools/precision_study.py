#!/usr/bin/env python
"""Accuracy and speed of the ResnetFC GEMM precision modes on one MI355X.

For N random points of the SRN scene, compares the HIP point query in each mode
("fp32" f32-MFMA, "bf16x9", "bf16x6" split-bf16 MFMA, "f16x3" scaled split-fp16) and the CPU fp32 oracle
against an fp64 evaluation of the same network (oracle/ref_cpu.py in double),
then times a cfg2 render chunk (4096 rays x (64 + 64)) per mode.
Prints one JSON object.
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from oracle import ref_cpu  # noqa: E402
from pnr import synth, util  # noqa: E402
from pnr.models import PixelNeRFNet  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402


def conf():
    mlp = dict(type="resnet", n_blocks=5, d_hidden=512, combine_layer=3, combine_type="average")
    return dict(use_encoder=True, use_xyz=True, use_code=True,
                code=dict(num_freqs=6, freq_factor=1.5), use_viewdirs=True,
                use_code_viewdirs=False, mlp_coarse=mlp, mlp_fine=mlp,
                encoder=dict(backbone="resnet34", pretrained=False, num_layers=4))


def main():
    dev = torch.device("cuda:0")
    n = int(os.environ.get("N_POINTS", "4096"))
    sd = synth.pixelnerf_state(1)
    lat = synth.latent(0, 1, 512, 64, 64)
    poses = synth.srn_poses([0.0])
    # points along real rays of the cfg2 frame (where the network is evaluated)
    rays = util.gen_rays(synth.srn_poses([30.0]), 128, 128, torch.tensor(131.25), 0.01, 4.0).reshape(-1, 8)
    idx = torch.from_numpy((synth.hash_uniform(5, n) * rays.shape[0]).astype("int64"))
    t = torch.from_numpy(synth.hash_uniform(6, n)).float()
    r = rays[idx]
    z = 0.8 + 1.0 * t
    xyz = (r[:, :3] + z[:, None] * r[:, 3:6])[None]
    vd = r[:, 3:6][None].contiguous()

    scene32 = ref_cpu.Scene(lat, poses, torch.tensor(131.25), 128, 128, None)
    sd64 = {k: v.double() for k, v in sd.items()}
    scene64 = ref_cpu.Scene(lat.double(), poses.double(), torch.tensor(131.25, dtype=torch.float64),
                            128, 128, None)
    scene64.poses = scene64.poses.double()
    scene64.focal = scene64.focal.double()
    scene64.c = scene64.c.double()
    scene64.image_shape = scene64.image_shape.double()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    res = {"n_points": n}
    with torch.no_grad():
        ref64 = ref_cpu.pixelnerf_forward(sd64, scene64, xyz.double(), True, vd.double())
        ref32 = ref_cpu.pixelnerf_forward(sd, scene32, xyz, True, vd)
    d = (ref32.double() - ref64).abs()
    res["oracle_fp32_vs_fp64"] = dict(max=float(d.max()), mean=float(d.mean()))

    net = PixelNeRFNet(conf())
    net.load_state_dict(sd, strict=False)
    net = net.to(dev).eval()
    net.encode_latent(lat.to(dev), poses.to(dev), torch.tensor(131.25, device=dev), (128, 128))
    frame = util.gen_rays(synth.srn_poses([30.0]), 128, 128, torch.tensor(131.25), 0.01, 4.0)
    chunk = frame.reshape(-1, 8)[:4096].to(dev)[None]
    for prec in ("fp32", "bf16x9", "bf16x6", "f16x3"):
        net.mlp_precision = prec
        with torch.no_grad():
            out = net(xyz.to(dev), coarse=True, viewdirs=vd.to(dev)).double().cpu()
        d = (out - ref64).abs()
        entry = dict(max=float(d.max()), mean=float(d.mean()),
                     max_vs_oracle32=float((out - ref32.double()).abs().max()))
        rr = NeRFRenderer(n_coarse=64, n_fine=64, white_bkgd=True)
        torch.manual_seed(0)
        with torch.no_grad():
            rr(net, chunk)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                rr(net, chunk)
            torch.cuda.synchronize()
        entry["chunk_ms"] = (time.perf_counter() - t0) / 3 * 1e3
        entry["rays_per_s"] = 4096 / (entry["chunk_ms"] * 1e-3)
        res[prec] = entry
    print(json.dumps(res))


if __name__ == "__main__":
    main()
