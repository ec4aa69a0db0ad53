"""Times the encoder trunk alone (conv1 .. layer3 + the channels-last latent, 4 x 3 x 128 x 128
SRN images) in three forms, for the training step (train-mode BN, forward + backward + Adam) and
for the render encode (eval mode, no grad):
    nchw           the shipped form (MIOpen convolutions, NCHW activations)
    channels_last  module and input in torch.channels_last (MIOpen's NHWC kernels)
    native         MIOpen disabled (torch.backends.cudnn.enabled = False: ATen's im2col + GEMM)
    python tools/encoder_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pixel-nerf_amd"))
from pnr.encoder import SpatialEncoder  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda:0")


def timed(fn, n=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for fmt in ("nchw", "channels_last", "native", "nchw", "channels_last", "native"):
    torch.backends.cudnn.enabled = fmt != "native"
    torch.manual_seed(0)
    enc = SpatialEncoder(pretrained=False).to(dev)
    x = torch.randn(4, 3, 128, 128, device=dev)
    if fmt == "channels_last":
        enc = enc.to(memory_format=torch.channels_last)
        x = x.contiguous(memory_format=torch.channels_last)
    opt = torch.optim.Adam(enc.parameters(), lr=1e-4)

    def step():
        opt.zero_grad(set_to_none=True)
        enc(x)
        (enc.latent_cl * 1e-3).sum().backward()
        opt.step()

    enc.train()
    t_train = timed(step)
    enc.eval()
    with torch.no_grad():
        t_enc = timed(lambda: enc(x))
    print("%-14s train step %.3f ms   eval encode %.3f ms" % (fmt, t_train, t_enc), flush=True)
torch.backends.cudnn.enabled = True
