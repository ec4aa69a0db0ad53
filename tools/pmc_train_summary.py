#!/usr/bin/env python
"""Per-kernel HBM bytes of the training step from tools/pmc_train.sh's two PMC passes: the mean
FETCH_SIZE (x2, the gfx950 correction for wide coalesced streaming reads, MI355X_MICROARCH.md)
and WRITE_SIZE per dispatch of the training MLP kernels, and the step totals (the last of the
two profiled steps: dispatches after the last FusedOptimizer launch of the warm-up)."""
import collections
import csv
import glob
import os
import sys


def rows(path):
    f = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    out = sys.argv[1]
    per = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        agg = collections.defaultdict(lambda: [0, 0.0])
        for r in rows(os.path.join(out, ctr)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if k.startswith("pnr::"):
                agg[k][0] += 1
                agg[k][1] += float(r["Counter_Value"])
        per[ctr] = agg
    print("# cfg5 training step (4 x 256 rays, 64 + 32 (16 depth)): HBM MB per dispatch of each pnr kernel, the")
    print("# mean over the profiled dispatches (warm-up + timed step: the same sizes); read = FETCH_SIZE x 2")
    print("# (gfx950 correction for wide coalesced streaming reads, MI355X_MICROARCH.md), write = WRITE_SIZE")
    print("kernel,dispatches,read_MB_per_dispatch,write_MB_per_dispatch")
    tot = [0.0, 0.0]
    for k in sorted(per["FETCH_SIZE"], key=lambda k: -per["FETCH_SIZE"][k][1]):
        n, f = per["FETCH_SIZE"][k]
        nw, w = per["WRITE_SIZE"].get(k, [n, 0.0])
        r_mb, w_mb = 2 * f / n / 1024, w / max(nw, 1) / 1024
        tot[0] += r_mb * n / 2
        tot[1] += w_mb * n / 2
        print('"%s",%d,%.1f,%.1f' % (k, n, r_mb, w_mb))
    print("per step (half the dispatches: warm-up + one timed step): read %.0f MB, write %.0f MB" % tuple(tot))


if __name__ == "__main__":
    main()
