#!/usr/bin/env python3
"""Per-basic-block instruction census of one kernel in a hipcc -S listing (gfx950):
  asm_blocks.py <file.s> <kernel-symbol-substring> [--min N]
For every block (.LBB label) of the kernel: MFMA, VALU, SALU, LDS, VMEM, waitcnt and branch counts, and the
branch targets, so the hot loop's body can be read off (the block whose count of MFMAs matches a pair step)."""
import argparse
import re
from collections import Counter


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op == "s_waitcnt":
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "br"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith(("s_barrier", "s_sched", "s_setprio")):
        return "sync"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--min", type=int, default=1, help="show blocks with at least this many instructions")
    ap.add_argument("--ops", action="store_true", help="list the VALU/SALU opcodes of each shown block")
    a = ap.parse_args()
    lines = open(a.asm).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and a.kernel in l)
    end = next((i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end")), len(lines))
    blocks, cur, name = [], [], "entry"
    for l in lines[start + 1:end]:
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            blocks.append((name, cur))
            name, cur = m.group(1), []
            continue
        s = l.strip()
        if not s or s.startswith((";", ".", "//")):
            continue
        cur.append(s.split(";")[0].strip())
    blocks.append((name, cur))
    tot = Counter()
    for name, ins in blocks:
        c = Counter(classify(x.split()[0]) for x in ins)
        tot += c
        if len(ins) < a.min:
            continue
        tg = [x.split()[1] for x in ins if x.split()[0].startswith(("s_cbranch", "s_branch"))]
        print(f"{name:14s} n={len(ins):4d} " + " ".join(f"{k}={c[k]}" for k in
              ("mfma", "valu", "salu", "lds", "vmem", "smem", "wait", "nop", "sync", "br") if c[k]) + f"  -> {tg}")
        if a.ops:
            ops = Counter(x.split()[0] for x in ins if classify(x.split()[0]) in ("valu", "salu"))
            print("     ", dict(ops.most_common()))
    print("total", dict(tot))


if __name__ == "__main__":
    main()
