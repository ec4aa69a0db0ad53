#!/usr/bin/env python
"""Mean PMC counter values of the k_point_mlp launches of one render pass in a rocprofv3
--pmc output (run_counter_collection.csv), passes labelled as scripts/summarize_profile.py does
(the sampler launched before an MLP launch names its pass).
Usage: tools/pmc_fine.py <dir with run_counter_collection.csv> [pass=fine]"""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
from summarize_profile import kname, pass_of  # noqa: E402


def main():
    d, want = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "fine")
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    by_disp = collections.OrderedDict()
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        e = by_disp.setdefault(r["Dispatch_Id"], {"name": kname(r["Kernel_Name"]), "ctr": collections.Counter(),
                                                  "ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6})
        e["ctr"][r["Counter_Name"]] += float(r["Counter_Value"])
    last, sel = "query", []
    for e in by_disp.values():
        n = e["name"]
        if "k_sample_coarse" in n:
            last = "coarse"
        elif "k_sample_fine" in n:
            last = "fine"
        elif "k_point_mlp" in n:
            if pass_of(n, last) == want:
                sel.append(e)
            last = "query"
    if not sel:
        print("no %s-pass k_point_mlp launches" % want)
        return
    ctr = collections.Counter()
    for e in sel:
        ctr.update(e["ctr"])
    ms = sum(e["ms"] for e in sel) / len(sel)
    out = ["%s pass: %d launches, %.3f ms" % (want, len(sel), ms)]
    for k in sorted(ctr):
        v = ctr[k] / len(sel)
        out.append("%s %.4g" % (k, v))
        if k == "FETCH_SIZE":
            out.append("hbm_gb(x2) %.3f" % (v * 2 * 1024e-9))
        if k == "GRBM_GUI_ACTIVE":
            out.append("clock_ghz %.3f" % (v / 8 / (ms * 1e6)))
    print("  ".join(out))


if __name__ == "__main__":
    main()
