#!/usr/bin/env python
"""Derived PMC metrics of the k_point_mlp launches from scripts/counters.sh output.

Usage: python scripts/analyze_counters.py gpurun_out/ctr_<tag> [kernel substring]
For k_point_mlp (default) per render pass (coarse / fine, told apart by launch order within
each probe chunk: coarse MLP first, then fine), for any other kernel over all its launches,
prints the mean over launches of:
  clock_ghz      GRBM_GUI_ACTIVE / XCDs / duration
  mfma_busy      SQ_VALU_MFMA_BUSY_CYCLES / (CUs * 4 SIMDs * clock cycles)
  wait_any, wait_inst, active_inst   SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY
                 as fractions of SQ_WAVE_CYCLES (MI355X_MICROARCH.md: disjoint, sum ~ 1)
  lds_conflict   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  l2_hit         TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  l2_req_gb      (TCC_HIT_sum + TCC_MISS_sum) x 128 B: L2 requests of the launch (CU reads
                 of 16 B/lane coalesced rows arrive as 128-B line requests)
  valu_active    SQ_ACTIVE_INST_VALU x 4 (quad-cycles) / (CUs * 4 SIMDs * clock cycles)
  hbm_gb         FETCH_SIZE x 2 (KB; gfx950 correction of MI355X_MICROARCH.md), when collected
"""
import csv
import glob
import os
import sys
from collections import defaultdict

CUS, XCDS = 256, 8


def load(d, kernel="k_point_mlp"):
    per = defaultdict(dict)   # dispatch id -> {counter: value, "name", "dur"}
    for path in glob.glob(os.path.join(d, "g*", "run_counter_collection.csv")):
        grp = os.path.basename(os.path.dirname(path))
        with open(path) as f:
            for r in csv.DictReader(f):
                if kernel not in r["Kernel_Name"]:
                    continue
                key = (grp, int(r["Dispatch_Id"]))
                e = per[key]
                e["name"] = r["Kernel_Name"].split("(")[0].replace("void ", "")
                e["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                e[r["Counter_Name"]] = float(r["Counter_Value"])
    # label passes: within each group, MLP launches alternate coarse, fine (probe chunks)
    out = defaultdict(lambda: defaultdict(list))
    for grp in sorted(set(k[0] for k in per)):
        ids = sorted(k[1] for k in per if k[0] == grp)
        for i, did in enumerate(ids):
            e = per[(grp, did)]
            label = ("%s %s" % (e["name"], "coarse" if i % 2 == 0 else "fine")
                     if kernel == "k_point_mlp" else e["name"])
            for k, v in e.items():
                if k != "name":
                    out[label][k].append(v)
    return out


def mean(v):
    return sum(v) / len(v) if v else float("nan")


def main():
    res = load(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_point_mlp")
    for label, c in sorted(res.items()):
        m = {k: mean(v) for k, v in c.items()}
        line = [label, "dur %.3f ms" % (m["dur"] * 1e3)]
        if "GRBM_GUI_ACTIVE" in m:
            clk = m["GRBM_GUI_ACTIVE"] / XCDS / m["dur"]
            line.append("clock %.2f GHz" % (clk / 1e9))
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                line.append("mfma_busy %.3f" % (m["SQ_VALU_MFMA_BUSY_CYCLES"] / (CUS * 4 * clk * m["dur"])))
        if "SQ_WAVE_CYCLES" in m:
            wc = m["SQ_WAVE_CYCLES"]
            for k, nm in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst"),
                          ("SQ_ACTIVE_INST_ANY", "active_inst")):
                if k in m:
                    line.append("%s %.3f" % (nm, m[k] / wc))
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            line.append("lds_conflict %.3f" % (m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]))
        if "TCC_HIT_sum" in m:
            line.append("l2_hit %.4f" % (m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])))
            line.append("l2_req_gb %.1f" % ((m["TCC_HIT_sum"] + m["TCC_MISS_sum"]) * 128e-9))
        if "FETCH_SIZE" in m:
            line.append("hbm_gb %.2f" % (m["FETCH_SIZE"] * 2 * 1024e-9))
        if "SQ_INSTS_VALU" in m and "SQ_INSTS_MFMA" in m:
            line.append("valu/mfma %.2f" % (m["SQ_INSTS_VALU"] / m["SQ_INSTS_MFMA"]))
        if "SQ_ACTIVE_INST_VALU" in m and "GRBM_GUI_ACTIVE" in m:
            # quad-cycles (MI355X_MICROARCH.md) of VALU issue, all waves, per SIMD cycle
            line.append("valu_active %.3f" % (m["SQ_ACTIVE_INST_VALU"] * 4 / (CUS * 4 * clk * m["dur"])))
        print("  ".join(line))


if __name__ == "__main__":
    main()
