"""Time pnr_weight_grad alone (diagnostic): 13 layers x P points (the fine pass of the
cfg5 training step: P = 1024 rays x 96 samples), HIP-event timed, fp32-equivalent TFLOP/s."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))
import torch  # noqa: E402

from pnr import train  # noqa: E402


def main():
    P = int(os.environ.get("P", 98304))
    J = int(os.environ.get("J", 13))
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    dys = [torch.randn(P, 512, device=dev, generator=g) * 1e-3 for _ in range(J)]
    xs = [torch.relu(torch.randn(P, 512, device=dev, generator=g)) for _ in range(J)]
    for _ in range(3):
        train.weight_grad(dys, xs, P)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record()
    for _ in range(n):
        train.weight_grad(dys, xs, P)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    flop = 2.0 * 512 * 512 * P * J
    print('{"P": %d, "layers": %d, "ms": %.3f, "tflops_fp32_equiv": %.1f}' % (P, J, ms, flop / ms / 1e9))


if __name__ == "__main__":
    main()
