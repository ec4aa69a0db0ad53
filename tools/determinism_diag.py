"""Diagnostic (GPU): point-query outputs of the in-tree libpnr.so against the fw_pointquery
fixture, repeated to separate a race (run-to-run differences) from a deterministic error, with
the bad points' tile / column.  Usage: python tools/determinism_diag.py [runs]  (PNR_LIB_PATH selects a variant build)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "tests"), os.path.join(REPO, "pixel-nerf_amd"), REPO):
    sys.path.insert(0, p)

import torch  # noqa: E402

import fixtures  # noqa: E402
from test_gpu_parity import close_mask, hip_net  # noqa: E402


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    cfg, arr = fixtures.load("fw_pointquery")
    for prec in ("f16x3",):
        net = hip_net(dict(cfg, n_blocks=5, combine_layer=3, with_fine=True, d_latent=512, d_hidden=512), arr,
                      prec, True)
        vd = torch.zeros_like(arr["xyz"]).cuda()
        for coarse in (True, False):
            ref = arr["out_coarse" if coarse else "out_fine"]
            outs = []
            with torch.no_grad():
                for _ in range(runs):
                    outs.append(net(arr["xyz"].cuda(), coarse=coarse, viewdirs=vd).cpu())
            same = all(torch.equal(outs[0], o) for o in outs[1:])
            for k, o in enumerate(outs):
                ok = close_mask(o, ref)
                bad = (~ok).reshape(-1, 4).any(-1).nonzero().flatten().tolist()
                d = (o - ref).abs().reshape(-1, 4).max(-1).values
                print("%s %s run %d: bad points %d %s  max|d| %.3g  deterministic %s" % (
                    prec, "coarse" if coarse else "fine", k, len(bad),
                    [(p, p // 64, p % 64, "%.2g" % float(d[p])) for p in bad[:24]], float(d.max()), same))


if __name__ == "__main__":
    main()
