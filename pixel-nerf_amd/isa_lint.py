#!/usr/bin/env python3
"""Build-time ISA lint for the gfx950 kernels ("the MARCH-kernel faults").

ROCm 7.2's AMDGPU backend can place a register spill or reload in a join block BEFORE the
block's EXEC restore (the ``s_or_b64 exec, exec, s[..]`` that ends a divergent ``if``).  The
spill then executes under the ``if``'s lane mask: only the lanes that took the branch write their
scratch slot, and the reload after the restore hands every other lane whatever the previous
user of that scratch slot left there.  Round 5's two unexplained ``hipErrorIllegalAddress``
faults were this: the thread id, spilled at the join of ``if (tid == 0) *s_next = grab();``,
came back as stale scratch and fed the sample / gather addresses
(k_point_mlp<6,true,true> in the 8299515 tree, <3,false,true> in d9605a6; the shipped tree had
no such spill).

The lint reads the device assembly that ``hipcc -save-temps=obj`` leaves for each object (the
same code as the library: the build is otherwise unchanged) and fails when, in any machine
basic block, a spill / reload (``scratch_*``, or an AGPR spill ``v_accvgpr_*``) comes before
the block's EXEC restore with no other EXEC write in between.  Usage:

    python3 isa_lint.py build/*.gfx950.s        (exit status 1 and a report on a hit)
"""
import re
import sys

_FUNC = re.compile(r"^([A-Za-z_.$][\w.$]*):")
_BLOCK = re.compile(r"^(\.LBB\w+:|\s*; %bb\.\d+:)")
_RESTORE = re.compile(r"^s_or_b64\s+exec,\s*exec,")
_EXEC_WRITE = re.compile(r"^s_\w+\s+exec\b|^s_\w*saveexec\w*\s")
_SPILL = re.compile(r"^(scratch_|v_accvgpr_(read|write)|buffer_(load|store)_\w+.*\boffen\b)")
# a whole-wave section (SGPR spills to VGPR lanes): s_or_saveexec_b64 s[..], -1 ... s_mov_b64 exec, s[..]
_WWM_ON = re.compile(r"^s_or_saveexec_b64\s+(s\[\d+:\d+\]),\s*-1\b")


def lint_file(path):
    """[(function, line number, instruction, restore)] of the spills placed before an EXEC restore."""
    hits = []
    fn = None
    pending = []      # spill / reload lines of the current block, before any EXEC write
    scanning = True   # no EXEC write seen yet in this block
    wwm = None        # inside a whole-wave section: the SGPR pair that restores EXEC
    with open(path) as f:
        for n, raw in enumerate(f, 1):
            m = _FUNC.match(raw)
            if m and not raw.startswith(".L"):
                fn, pending, scanning, wwm = m.group(1), [], True, None
                continue
            if _BLOCK.match(raw):
                pending, scanning, wwm = [], True, None
                continue
            ins = raw.split(";")[0].strip()
            if not ins or ins.startswith("."):
                continue
            if not scanning:
                continue
            if wwm is not None:   # whole-wave spills are correct under any mask: skip the section
                if re.match(r"^s_mov_b64\s+exec,\s*" + re.escape(wwm) + r"$", ins):
                    wwm = None
                continue
            w = _WWM_ON.match(ins)
            if w:
                wwm = w.group(1)
                continue
            if _RESTORE.match(ins):
                hits += [(fn, ln, s, ins) for ln, s in pending]
                pending, scanning = [], False
            elif _EXEC_WRITE.match(ins):
                pending, scanning = [], False
            elif _SPILL.match(ins):
                pending.append((n, ins))
    return hits


def main(paths):
    bad = 0
    for p in paths:
        for fn, ln, ins, restore in lint_file(p):
            bad += 1
            print("%s:%d: %s: spill/reload '%s' executes under a branch's lane mask "
                  "(before '%s')" % (p, ln, fn, ins, restore), file=sys.stderr)
    if bad:
        print("isa_lint: %d spill(s) before an EXEC restore: this build would hand stale scratch "
              "to inactive lanes (see isa_lint.py)" % bad, file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
