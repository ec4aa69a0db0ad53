"""Retune counts of k_wgrad_h (the f16x3 weight gradient's scale moves, csrc/wgrad.hip) on the
training step's own data: runs bench.train_leg with a -DPNR_WGH_STATS build and reads its counters.
    scripts/build_variant.sh wgh_stats WORKTREE -DPNR_WGH_STATS
    PNR_LIB_PATH=pixel-nerf_amd/build/wgh_stats/libpnr.so python tools/wgrad_stats.py"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from pnr import _lib  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
lib = _lib.load()
lib.pnr_wgrad_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
st = (ctypes.c_ulonglong * 5)()
bench.train_leg(dev, 0, 1, 2, 1, precision="f16x3", sb=4, per=256, ns=1, graph=False, sync_debug=False)
assert lib.pnr_wgrad_stats(st, 1) == 0
print("training steps (3): retunes after step 0 %d over %d steps in %d workgroups (%.2f %% of steps)"
      % (st[0], st[1], st[2], 100.0 * st[0] / max(st[1], 1)))
print("  channel scale moves after step 0: %d from unset, %d by growth" % (st[3], st[4]))
P = 65536
g = torch.Generator(device=dev).manual_seed(0)
dys = [torch.randn(P, 512, device=dev, generator=g) for _ in range(13)]
xs = [torch.relu(torch.randn(P, 512, device=dev, generator=g)) for _ in range(13)]
from pnr import train  # noqa: E402
train.weight_grad(dys, xs, P)
assert lib.pnr_wgrad_stats(st, 1) == 0
print("gaussian probe: retunes %d over %d steps in %d workgroups" % (st[0], st[1], st[2]))
