"""Times the encoder trunk's training work alone (forward + backward of conv1 .. layer3 + the
channels-last latent, 4 x 3 x 128 x 128 SRN images) in NCHW and in channels_last memory format.
    python tools/encoder_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pixel-nerf_amd"))
from pnr.encoder import SpatialEncoder  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda:0")
for fmt in ("nchw", "channels_last", "nchw", "channels_last"):
    torch.manual_seed(0)
    enc = SpatialEncoder(pretrained=False).to(dev)
    x = torch.randn(4, 3, 128, 128, device=dev)
    if fmt == "channels_last":
        enc = enc.to(memory_format=torch.channels_last)
        x = x.contiguous(memory_format=torch.channels_last)
    opt = torch.optim.Adam(enc.parameters(), lr=1e-4)

    def step():
        opt.zero_grad(set_to_none=True)
        lat = enc(x)
        (enc.latent_cl * 1e-3).sum().backward()
        opt.step()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        step()
    e1.record()
    torch.cuda.synchronize()
    print("%-14s %.3f ms per step" % (fmt, e0.elapsed_time(e1) / 20))
