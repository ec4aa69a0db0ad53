"""Smallest |ReLU input| among units that carry gradient in the oracle's training step
(diagnostic for the gradient tests: a unit within fp32 rounding of zero can land on the
other side of the kink in another fp32 evaluation and move every gradient below it).

  python tools/relu_margin.py [ns] [seed] [--conditioned]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pixel-nerf_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

import test_gpu_train as t  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    ns = int(args[0]) if args else 2
    seed = int(args[1]) if len(args) > 1 else 3
    torch.set_num_threads(8)
    cs = t.case(ns=ns, seed=seed)
    if "--conditioned" in sys.argv:
        cs["sd"] = t.conditioned(cs["sd"])
    orig = torch.relu
    recs = []

    def relu(x):
        y = orig(x)
        if y.requires_grad:
            y.retain_grad()
            recs.append((x.detach(), y))
        return y

    torch.relu = relu
    try:
        loss, g = t.oracle_grads(cs)
    finally:
        torch.relu = orig
    margin = float("inf")
    for x, y in recs:
        if y.grad is None:
            continue
        live = (y.grad.abs() > 0) & (x != 0)
        if live.any():
            margin = min(margin, float(x.abs()[live].min()))
    print("ns %d seed %d loss %.6g  min |relu input| carrying gradient %.3g" % (ns, seed, loss, margin))
    for k in sorted(g):
        if "blocks.2" in k or k == "latent":
            print("  max |grad| %-36s %.3g" % (k, float(g[k].abs().max())))


if __name__ == "__main__":
    main()
