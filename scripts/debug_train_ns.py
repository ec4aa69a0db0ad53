"""Per-tensor gradient error of the HIP training step vs the oracle (diagnostic)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "pixel-nerf_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

import test_gpu_train as t  # noqa: E402

torch.set_num_threads(8)
for ns, kfd, seed in [(1, 0, 11), (2, 0, 3)]:
    for prec in ["fp32", "f16x3", "fp32"]:
        cs = t.case(ns=ns, kfd=kfd, kf=24 if kfd else 16, seed=seed)
        rl, ref = t.oracle_grads(cs)
        l, got = t.hip_grads(cs, prec)
        errs = []
        for k in sorted(ref):
            a, b = got[k].reshape(-1).double(), ref[k].reshape(-1).double()
            errs.append((float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30), k))
        errs.sort()
        print("ns", ns, "kfd", kfd, prec, "loss rel %.2g" % (abs(l - rl) / rl), "worst:",
              flush=True)
        for e, k in errs[-5:]:
            print("   %-40s %.3g" % (k, e))
