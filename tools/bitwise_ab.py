#!/usr/bin/env python
"""Diagnostic (GPU): is a libpnr.so variant bit-identical to another on the bench's cfg3 render?
Renders the first 8,192 rays of the cfg3 batch (64 + 64, counter RNG with a fixed seed, a synthetic
32 x 32 latent) with the library PNR_LIB_PATH selects and saves coarse / fine rgb, depth and weights.

  python tools/bitwise_ab.py save OUT.pt        (run once per variant, each in its own process)
  python tools/bitwise_ab.py cmp A.pt B.pt      (CPU: bitwise equal? max |diff| otherwise)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def save(out):
    import torch

    import bench
    from pnr.renderer import NeRFRenderer

    from pnr import synth

    dev = torch.device("cuda:0")
    net = bench.make_net(dev, "f16x3", True, use_first_pool=False)
    img, src, focal, rays = bench.nmr_inputs(dev)
    r = NeRFRenderer(n_coarse=bench.KC, n_fine=bench.KF, white_bkgd=True).to(dev)
    with torch.no_grad():
        # a synthetic latent, not the ResNet34 encode: MIOpen may pick another convolution
        # algorithm in another process, which changes the latent in its last bits
        net.encode_latent(synth.latent(0, 1, 512, 32, 32).to(dev), src, focal, (64, 64))
        torch.manual_seed(7)
        d = r(net, rays[:8192][None], want_weights=True)
    torch.save({f"{p}.{k}": d[p][k].cpu() for p in ("coarse", "fine") for k in ("rgb", "depth", "weights")}, out)
    print("saved", out, os.environ.get("PNR_LIB_PATH", "default"))


def cmp(a, b):
    import torch

    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    same = True
    for k in A:
        eq = torch.equal(A[k], B[k])
        same &= eq
        print(k, "identical" if eq else "max|d| %.3e" % float((A[k] - B[k]).abs().max()))
    print("BITWISE IDENTICAL" if same else "DIFFERENT")
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(save(sys.argv[2]) if sys.argv[1] == "save" else cmp(sys.argv[2], sys.argv[3]))
