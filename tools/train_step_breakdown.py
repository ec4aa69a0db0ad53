"""Per-kernel time of the LAST training step in a rocprofv3 kernel trace of
scripts/bench_train.py (the step after the last-but-one fine-MLP backward).
Usage: python tools/train_step_breakdown.py <run_kernel_trace.csv> [top]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # two MLP launches per step (coarse, fine); the backward kernel marks the step tail
    marks = [i for i, r in enumerate(rows) if "k_mlp_bwd" in r["Kernel_Name"]]
    if len(marks) < 4:
        marks = [i for i, r in enumerate(rows) if "k_point_mlp" in r["Kernel_Name"]]
    seg = rows[marks[-3] + 1: marks[-1] + 1]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in seg:
        k = r["Kernel_Name"]
        k = k[5:] if k.startswith("void ") else k
        tot[k[:110]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        cnt[k[:110]] += 1
    print("one step: span %.3f ms, kernel busy %.3f ms, %d dispatches" % ((t1 - t0) / 1e6, sum(tot.values()) / 1e6,
                                                                        len(seg)))
    for k, v in sorted(tot.items(), key=lambda x: -x[1])[:top]:
        print("%8.3f ms %4d  %s" % (v / 1e6, cnt[k], k))
    # idle gaps: time between a kernel's end and the next kernel's start (host-bound stretches)
    gaps = []
    end = int(seg[0]["End_Timestamp"])
    for prev, r in zip(seg, seg[1:]):
        st = int(r["Start_Timestamp"])
        if st > end:
            gaps.append((st - end, prev["Kernel_Name"][:60], r["Kernel_Name"][:60]))
        end = max(end, int(r["End_Timestamp"]))
    gaps.sort(reverse=True)
    print("idle total %.3f ms in %d gaps; largest:" % (sum(g[0] for g in gaps) / 1e6, len(gaps)))
    for g in gaps[:12]:
        print("  %7.3f ms  after %s  before %s" % (g[0] / 1e6, g[1], g[2]))

    phases(rows)


def phases(rows):
    """Wall span and kernel-busy time of the step's regions, delimited by landmark kernels: the
    step is the dispatches after the last-but-one Adam (FusedOptimizer) kernel group up to the last
    one; regions end at the first coarse / fine forward MLP, the first / second k_mlp_bwd, the
    last k_points_in_bwd and the first Adam kernel."""
    opt = [i for i, r in enumerate(rows) if "FusedOptimizer" in r["Kernel_Name"]]
    if len(opt) < 2:
        return
    # last Adam group: consecutive optimizer dispatches at the end
    last = opt[-1]
    first_of_last = last
    while first_of_last - 1 in opt:
        first_of_last -= 1
    prev = max(i for i in opt if i < first_of_last)
    seg = rows[prev + 1: last + 1]
    names = [r["Kernel_Name"] for r in seg]
    fwd = [i for i, n in enumerate(names) if "k_point_mlp" in n]
    bwd = [i for i, n in enumerate(names) if "k_mlp_bwd" in n]
    pin = [i for i, n in enumerate(names) if "k_points_in_bwd" in n]
    adam = [i for i, n in enumerate(names) if "FusedOptimizer" in n]
    if len(fwd) < 2 or len(bwd) < 2 or not pin or not adam:
        return
    cuts = [("encode (+ coarse draws)", fwd[0]), ("coarse forward MLP", fwd[0] + 1),
            ("fine draws", fwd[1]), ("fine forward MLP", fwd[1] + 1),
            ("loss + composite backward", bwd[0]), ("first MLP backward (+ wgrad, input bwd)", bwd[1]),
            ("second MLP backward (+ wgrad, input bwd)", pin[-1] + 1),
            ("encoder backward + grad glue", adam[0]), ("Adam", len(seg))]
    print("step regions (wall span incl. idle / kernel busy):")
    lo = 0
    t_prev_end = int(seg[0]["Start_Timestamp"])
    for name, hi in cuts:
        part = seg[lo:hi]
        if part:
            t0 = t_prev_end
            t1 = max(int(r["End_Timestamp"]) for r in part)
            busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in part)
            print("  %-44s %7.3f ms  busy %7.3f ms  %4d dispatches" % (name, (t1 - t0) / 1e6, busy / 1e6, len(part)))
            t_prev_end = t1
        lo = hi


if __name__ == "__main__":
    main()
