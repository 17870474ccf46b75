#!/usr/bin/env python3
"""Dev tool: per-basic-block instruction mix of one kernel in a hipcc -S (.s) file.

usage: isa_blocks.py FILE.s KERNEL_REGEX [--min N] [--grep OPCODE_REGEX]
Prints, for every block of the first kernel whose symbol matches, its label and counts of VALU
(v_*), SALU (s_* except branches/waits), LDS (ds_*), VMEM (global_/buffer_), waits and branches;
blocks containing an instruction matching --grep are starred (e.g. 'v_alignbit' marks the step).
"""
import argparse
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("kernel")
    ap.add_argument("--min", type=int, default=8, help="hide blocks with fewer instructions")
    ap.add_argument("--grep", default=r"v_alignbit")
    args = ap.parse_args()
    lines = open(args.path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        m = re.match(r"^(\S+):\s*(;.*)?$", l)
        if m and m.group(1).startswith("_Z") and re.search(args.kernel, m.group(1)):
            start = i
            name = m.group(1)
            break
    if start is None:
        raise SystemExit("kernel not found")
    print(name)
    blocks, cur, label = [], [], "entry"
    for l in lines[start + 1 :]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            blocks.append((label, cur))
            label, cur = m.group(1), []
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")):
            continue
        cur.append(s.split()[0])
    blocks.append((label, cur))
    tot = {"valu": 0, "salu": 0, "lds": 0, "vmem": 0}
    for label, ins in blocks:
        c = {"valu": 0, "salu": 0, "lds": 0, "vmem": 0, "wait": 0, "br": 0}
        for op in ins:
            if op.startswith("v_"):
                c["valu"] += 1
            elif op.startswith("ds_"):
                c["lds"] += 1
            elif op.startswith(("global_", "buffer_", "flat_")):
                c["vmem"] += 1
            elif op.startswith("s_waitcnt"):
                c["wait"] += 1
            elif op.startswith(("s_cbranch", "s_branch")):
                c["br"] += 1
            elif op.startswith("s_"):
                c["salu"] += 1
        for k in tot:
            tot[k] += c[k]
        if len(ins) >= args.min:
            star = "*" if any(re.match(args.grep, op) for op in ins) else " "
            print(f"{star} {label:14s} n={len(ins):4d} valu={c['valu']:4d} salu={c['salu']:3d} lds={c['lds']:3d} "
                  f"vmem={c['vmem']:3d} wait={c['wait']:3d} br={c['br']:2d}")
    print("total", tot)


if __name__ == "__main__":
    main()
