#!/usr/bin/env python
"""Mean counters of the save probe's k_point_mlp dispatches (tools/save_counters_probe.py): the
first half WITH the activation save, the second half WITHOUT; one line each, from the counter
CSVs of scripts/counters.sh-style passes.  Usage: tools/save_counters.py <dir> [<dir> ...]"""
import collections
import csv
import glob
import os
import sys

tot = {"save": collections.Counter(), "no save": collections.Counter()}
dur = {"save": [], "no save": []}
for d in sys.argv[1:]:
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    disp = collections.OrderedDict()
    for r in csv.DictReader(open(f[0])):
        if "k_point_mlp" not in r["Kernel_Name"]:
            continue
        e = disp.setdefault(int(r["Dispatch_Id"]), [collections.Counter(),
                                                     (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6])
        e[0][r["Counter_Name"]] += float(r["Counter_Value"])
    ids = sorted(disp)
    half = len(ids) // 2
    for i, k in enumerate(ids):
        tag = "save" if i < half else "no save"
        for c, v in disp[k][0].items():
            tot[tag][c] += v / half
        dur[tag].append(disp[k][1])
for tag in ("save", "no save"):
    c = tot[tag]
    ms = sum(dur[tag]) / max(len(dur[tag]), 1)
    line = ["%-8s dur %.3f ms" % (tag, ms)]
    for k in sorted(c):
        line.append("%s %.4g" % (k, c[k]))
    print("  ".join(line))
