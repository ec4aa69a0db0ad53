#!/usr/bin/env python
"""Summarize a scripts/profile.sh run (gpurun_out/prof_<tag>) into profiles/<tag>/.

  kernel_stats.csv  rocprofv3 --kernel-trace --stats summary (copied as is)
  pmc_summary.csv   per-dispatch FETCH_SIZE / WRITE_SIZE (KB, as rocprofv3 reports them)
                    and the HBM bytes with the gfx950 correction of MI355X_MICROARCH.md
                    (FETCH_SIZE counts half of wide coalesced streaming reads: x2)

Usage: python scripts/summarize_profile.py <tag> [note] [workload]
(workload labels the PMC rows: the PMC passes of scripts/profile.sh run the cfg3 leg only)
"""
import csv
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def read_counter(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append(r)
    return rows


def pass_of(name, last):
    """Render pass of a k_point_mlp launch: the sampler launched before it names it; the fused
    march instantiation (k_point_mlp<P, Z, true>) draws its coarse depths itself, so one with
    no sampler before it is a coarse pass (pnr_render_set_fused mode 2)."""
    if last == "query" and name.replace(" ", "").endswith(",true>"):
        return "coarse"
    return last


def kname(full):
    """'void pnr::mlpk::k_point_mlp<3>(pnr::mlpk::Args)' -> 'pnr::mlpk::k_point_mlp<3>'"""
    n = full.split("(")[0].strip()
    return n[5:] if n.startswith("void ") else n


def trace_stats(src, dst):
    """kernel_stats.csv (as rocprofv3 wrote it) and the k_point_mlp launches by render pass."""
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    # per-dispatch MLP durations from the kernel trace, labelled by the sampling kernel
    # that precedes them in stream order (coarse / fine pass of pnr_render_forward)
    trace = read_counter(os.path.join(src, "trace", "run_kernel_trace.csv"))
    trace.sort(key=lambda r: int(r["Dispatch_Id"]))
    rows, last = [], "query"
    for r in trace:
        name = kname(r["Kernel_Name"])
        if "k_sample_coarse" in name:
            last = "coarse"
        elif "k_sample_fine" in name:
            last = "fine"
        elif "k_point_mlp" in name:
            ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
            rows.append((name, pass_of(name, last), ms))
            last = "query"
    stats = ["kernel,pass,launches,avg_ms,min_ms,max_ms"]
    for key in sorted(set((n, p) for n, p, _ in rows)):
        d = [ms for n, p, ms in rows if (n, p) == key]
        stats.append('"%s",%s,%d,%.4f,%.4f,%.4f' % (key[0], key[1], len(d), sum(d) / len(d), min(d), max(d)))
    with open(os.path.join(dst, "mlp_dispatch_stats.csv"), "w") as f:
        f.write("# k_point_mlp launches of the kernel-trace run, by render pass\n" + "\n".join(stats) + "\n")


def main():
    tag = sys.argv[1]
    note = sys.argv[2] if len(sys.argv) > 2 else ""
    workload = sys.argv[3] if len(sys.argv) > 3 else "cfg3"
    src = os.path.join(REPO, "gpurun_out", "prof_" + tag)
    # PNR_PROFILE_DST: write the summary elsewhere (on the GPU box, under gpurun_out/ so the same
    # lease's bench can read it with --traffic-from and it merges back; scripts/gpu_session.sh)
    dst = os.environ.get("PNR_PROFILE_DST") or os.path.join(REPO, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    fetch = read_counter(os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv"))
    write = read_counter(os.path.join(src, "pmc_WRITE_SIZE", "run_counter_collection.csv"))
    wmap = {r["Dispatch_Id"]: float(r["Counter_Value"]) for r in write}
    if os.path.exists(os.path.join(src, "trace", "run_kernel_stats.csv")):
        trace_stats(src, dst)
    lines = [
        "# rocprofv3 PMC summary, %s (bench.py cfg3 headline leg + the 1 M-ray composite leg, --steps 1 --warmup 0) %s" % (tag, note),
        "# FETCH_SIZE/WRITE_SIZE in KB as rocprofv3 reports them (per dispatch).",
        "# gfx950: FETCH_SIZE reads 1/2 of wide coalesced streaming reads (MI355X_MICROARCH.md HBM)"
        " -> corrected = 2x.",
        "kernel,grid,dispatch_ms,FETCH_SIZE_KB,WRITE_SIZE_KB,hbm_bytes_corrected,pass,workload   (kernel names quoted)",
    ]
    fetch.sort(key=lambda r: int(r["Dispatch_Id"]))
    last = "query"
    for r in fetch:
        name = kname(r["Kernel_Name"])
        if not name.startswith("pnr::"):
            continue
        if "k_sample_coarse" in name:
            last = "coarse"
        elif "k_sample_fine" in name:
            last = "fine"
        label, wl = "", workload
        fk = float(r["Counter_Value"])
        wk = wmap.get(r["Dispatch_Id"], 0.0)
        if "k_point_mlp" in name:
            label, last = pass_of(name, last), "query"
        elif "k_composite" in name and int(r["Grid_Size"]) >= (1 << 20) * 64 // 4:
            # bench.py composite_roofline: 1 M rays x 128 samples, without then with the weights
            # output (the weights add 512 B per ray of writes: 512 MB against 16 MB)
            wl, label = "composite_1M", ("weights" if wk > 256 * 1024 else "no_weights")
        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        lines.append('"%s",%s,%.4f,%.1f,%.1f,%d,%s,%s' % (name, r["Grid_Size"], ms, fk, wk,
                                                        int((2 * fk + wk) * 1024), label, wl))
    with open(os.path.join(dst, "pmc_summary.csv"), "w") as f:
        f.write("\n".join(lines) + "\n")
    clock_csv(src, dst)
    print("wrote", dst)


def clock_csv(src, dst):
    """Effective clock per k_point_mlp launch from a GRBM_GUI_ACTIVE pass (MI355X_MICROARCH.md
    "DVFS give-back": GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall time; within 3 % of the in-kernel
    clock on dispatches of 10 ms or more).  Note: the PMC pass serializes dispatches, so the
    launch runs without its neighbours' overlap, as in the bench."""
    path = os.path.join(src, "pmc_GRBM_GUI_ACTIVE", "run_counter_collection.csv")
    if not os.path.exists(path):
        return
    rows = read_counter(path)
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    out = ["# effective GPU clock per dispatch: GRBM_GUI_ACTIVE / 8 / dispatch time (MHz)",
           "kernel,pass,dispatch_ms,grbm_gui_active,mhz"]
    last = "query"
    for r in rows:
        name = kname(r["Kernel_Name"])
        if "k_sample_coarse" in name:
            last = "coarse"
        elif "k_sample_fine" in name:
            last = "fine"
        if "k_point_mlp" not in name and "k_composite" not in name:
            continue
        label = ""
        if "k_point_mlp" in name:
            label, last = pass_of(name, last), "query"
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        v = float(r["Counter_Value"])
        out.append('"%s",%s,%.4f,%d,%.1f' % (name, label, ns * 1e-6, v, v / 8 / (ns * 1e-9) / 1e6))
    with open(os.path.join(dst, "clock.csv"), "w") as f:
        f.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
