#!/usr/bin/env python
"""Numerical check of the loaded libpnr.so's standalone composite (PNR_LIB_PATH selects a variant)
against a torch float64 restatement of nerf.py:225-247 on random rays: max |d| of rgb / depth /
weights over K in {32, 64, 100, 128, 192}, white and black background."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))
import torch  # noqa: E402

from pnr import ops  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
worst = 0.0
for K in (32, 64, 100, 128, 192):
    for white in (True, False):
        B = 4099
        rays = torch.zeros(B, 8, device=dev)
        rays[:, 6], rays[:, 7] = 0.01, 4.0
        z = torch.sort(torch.rand(B, K, device=dev, generator=g) * 3.9 + 0.05, -1)[0]
        raw = torch.rand(B, K, 4, device=dev, generator=g)
        raw[..., 3] = raw[..., 3] * 8 - 2
        w, rgb, depth = ops.composite(z, raw, rays, white, want_weights=True)
        zd, rd = z.double(), raw.double()
        delta = torch.cat([zd[:, 1:] - zd[:, :-1], 4.0 - zd[:, -1:]], -1)
        alpha = 1 - torch.exp(-delta * torch.relu(rd[..., 3]))
        T = torch.cumprod(torch.cat([torch.ones_like(alpha[:, :1]), 1 - alpha + 1e-10], -1), -1)[:, :-1]
        wr = alpha * T
        rgbr = (wr[..., None] * rd[..., :3]).sum(1) + ((1 - wr.sum(1))[:, None] if white else 0)
        dr = (wr * zd).sum(1)
        e = max(float((w.double() - wr).abs().max()), float((rgb.double() - rgbr).abs().max()),
                float((depth.double() - dr).abs().max()))
        worst = max(worst, e)
        print("K %3d white %d: max |d| %.3g" % (K, white, e))
print("worst %.3g (%s)" % (worst, "ok" if worst < 5e-5 else "FAIL"))
