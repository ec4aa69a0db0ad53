#!/usr/bin/env python3
"""HBM bytes per k_point_mlp launch of the cfg4 DTU frame (tools/cfg4_probe.py) from a
rocprofv3 FETCH_SIZE pass, by render pass ("PMC FETCH bytes per launch").

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -o run -- python tools/cfg4_probe.py
  python tools/pmc_cfg4.py <dir>/.../run_counter_collection.csv [label]

In the fused march (mode 2) a chunk is: k_point_mlp (coarse pass, draws in its prologue),
k_sample_fine, k_point_mlp (fine pass); the first frame is the probe's warm-up.  FETCH_SIZE is
reported in KB; gfx950 counts half of wide coalesced streaming reads (MI355X_MICROARCH.md HBM),
so the corrected figure is 2x (as scripts/summarize_profile.py).  Prints one JSON object."""
import csv
import json
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    label = sys.argv[2] if len(sys.argv) > 2 else ""
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    prev, out = "", {"coarse": [], "fine": []}
    for r in rows:
        name = r["Kernel_Name"]
        if "k_point_mlp" in name:
            p = "fine" if "k_sample_fine" in prev else "coarse"
            out[p].append((float(r["Counter_Value"]), int(r["Grid_Size"])))
        if "pnr::" in name:
            prev = name
    res = {"label": label}
    for p, v in out.items():
        kb = [x for x, _ in v]
        res[p] = {"launches": len(kb), "fetch_kb_per_launch": [round(x) for x in kb],
                  "hbm_gb_per_launch_corrected_mean": round(2 * sum(kb) * 1024 / max(len(kb), 1) / 1e9, 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
