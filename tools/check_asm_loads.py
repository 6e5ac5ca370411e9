#!/usr/bin/env python3
"""Check hand-counted inline-asm loads in a gfx950 .s file (qfs_body.h).

qfs_body's raw sums and calibration are loaded by inline asm the compiler
cannot see, and waited for by a counted s_waitcnt vmcnt(N).  Nothing may read,
copy or spill those registers before such a wait covers the load.  For every
asm load, this walks forward to the first instruction that names one of its
destination registers and checks that some s_waitcnt vmcnt(N) in between has
at least N vector-memory instructions issued after the load and before it.
Forward branches in between are walked linearly; a backward one is reported.

usage: check_asm_loads.py file.s [kernel-symbol-substring]
"""
import re
import sys

VMEM = re.compile(r"^\s*(global_|buffer_|scratch_|flat_)\w+")
WAIT = re.compile(r"s_waitcnt\s+vmcnt\((\d+)\)")
REG = re.compile(r"v\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def main():
    lines = open(sys.argv[1]).read().split("\n")
    want = sys.argv[2] if len(sys.argv) > 2 else "mh_step_kernel"
    bad = review = checked = 0
    in_kernel = False
    in_asm = False
    for i, ln in enumerate(lines):
        if re.match(r"^_Z\S*:", ln):
            in_kernel = want in ln
        if not in_kernel:
            continue
        if ";;#ASMSTART" in ln:
            in_asm = True
            continue
        if ";;#ASMEND" in ln:
            in_asm = False
            continue
        if not (in_asm and re.match(r"^\s*global_load_dwordx[24]\s", ln)):
            continue
        dst = regs(ln.split(",")[0])
        checked += 1
        after = 0              # VMEM instructions issued after this load
        covered = False
        for k in range(i + 1, len(lines)):
            t = lines[k].split(";")[0]
            if not t.strip():
                continue
            w = WAIT.search(t)
            if w and after >= int(w.group(1)):
                covered = True
            if re.match(r"^\.LBB|^\s*s_(c?branch|setpc)", t) and not covered:
                # forward branches (the X DMA's if / else) are walked linearly, both arms
                # in turn; a backward branch ends the walk for review
                m = re.search(r"(\.LBB\d+_\d+)", t)
                if m and not t.startswith(".LBB") and any(l.startswith(m.group(1) + ":") for l in lines[i:k]):
                    print(f"review: line {i + 1}: backward branch at line {k + 1} before a covering wait")
                    review += 1
                    break
            if VMEM.match(t):
                after += 1
                if not covered and regs(t.split(",")[0]) & dst:
                    pass   # another load writing the same registers (reissue): fine only once covered
            if not w and regs(t) & dst and not VMEM.match(t):
                if not covered:
                    print(f"BAD: line {i + 1} ({ln.strip()}): line {k + 1} uses its registers first: {t.strip()}")
                    bad += 1
                break
            if VMEM.match(t) and regs(t) & dst and not covered:
                print(f"BAD: line {i + 1}: line {k + 1} touches its registers first: {t.strip()}")
                bad += 1
                break
    print(f"{checked} asm loads checked, {bad} bad, {review} to review")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
