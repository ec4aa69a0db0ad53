"""Times pnr_weight_grad (k_wgrad + k_wgrad_reduce) alone: 13 layers of 512 x 512 over P points,
the coarse training MLP's shape.  Select a libpnr.so variant with PNR_LIB_PATH.
    python tools/wgrad_probe.py [P] [jobs]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pixel-nerf_amd"))
from pnr import train  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
J = int(sys.argv[2]) if len(sys.argv) > 2 else 13
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
dys = [torch.randn(P, 512, device=dev, generator=g) for _ in range(J)]
xs = [torch.relu(torch.randn(P, 512, device=dev, generator=g)) for _ in range(J)]
for _ in range(3):
    train.weight_grad(dys, xs, P)
torch.cuda.synchronize()
n = 20
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(n):
    train.weight_grad(dys, xs, P)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / n
fl = 2.0 * J * 512 * 512 * P
print("P=%d jobs=%d: %.3f ms  %.1f fp32-equivalent TFLOP/s" % (P, J, ms, fl / ms / 1e9))
