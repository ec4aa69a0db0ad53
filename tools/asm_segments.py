#!/usr/bin/env python3
"""Per-barrier instruction counts of one kernel in `make -C pixel-nerf_amd asm` output
(build/mlp.s): a quick static check of what a code change does to the VALU / LDS / MFMA mix
of each phase between two s_barrier.  Usage: tools/asm_segments.py [kernel-symbol-substring]"""
import collections
import re
import sys

ASM = "pixel-nerf_amd/build/mlp.s"
want = sys.argv[1] if len(sys.argv) > 1 else "k_point_mlpILi3ELb1ELb1E"
lines = open(ASM).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(want), l))
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".end_amdhsa_kernel")
           or lines[i].strip() == "s_endpgm" and False) if False else None
end = next(i for i in range(start + 1, len(lines)) if re.match(r"^\s*\.Lfunc_end", lines[i]))
segs, cur, s0 = [], collections.Counter(), start
total = collections.Counter()
for i in range(start, end):
    t = lines[i].strip()
    if not t or t.startswith((";", ".")) or t.endswith(":"):
        continue
    op = t.split()[0]
    cur[op] += 1
    total[op] += 1
    if op == "s_barrier":
        segs.append((s0, i, cur))
        cur, s0 = collections.Counter(), i
segs.append((s0, end, cur))


def row(a, b, c):
    valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
    mx = sum(v for k, v in c.items() if k.startswith(("v_max", "v_maximum")))
    return ("%6d-%6d tot %5d mfma %4d valu %5d max %4d pkmul %3d dsw %3d dsr %3d gl %3d bperm %3d "
            "permlane %2d nop %3d" % (a, b, sum(c.values()), sum(v for k, v in c.items() if k.startswith("v_mfma")),
                                     valu, mx, c["v_pk_mul_f32"],
                                     sum(v for k, v in c.items() if k.startswith("ds_write")),
                                     sum(v for k, v in c.items() if k.startswith("ds_read")),
                                     sum(v for k, v in c.items() if k.startswith("global_load")),
                                     c["ds_bpermute_b32"],
                                     sum(v for k, v in c.items() if "permlane" in k), c["s_nop"]))


for a, b, c in segs:
    print(row(a, b, c))
print("TOTAL", row(start, end, total))
