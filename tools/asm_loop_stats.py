#!/usr/bin/env python3
"""Instruction mix of the hottest loop of one kernel in a hipcc -S listing:
finds the kernel's basic blocks, takes the largest block range closed by a backward
branch, and counts MFMA / VALU / v_mov / DS / VMEM / SALU / waits in it.
usage: asm_loop_stats.py file.s kernel_symbol_substring"""
import collections
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.split(";")[0].rstrip().endswith(":") and sym in l and not l.startswith("."))
end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
body = lines[start:end]
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
cands = []
for i, l in enumerate(body):
    m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\w+)|\s+s_branch\s+(\.LBB\w+)", l)
    if m:
        tgt = m.group(1) or m.group(2)
        if tgt in labels and labels[tgt] < i:
            n = sum("mfma" in x for x in body[labels[tgt]:i])
            if n >= int(__import__("os").environ.get("MIN_MFMA", "32")):
                cands.append((i - labels[tgt], labels[tgt], i))
# innermost loop that carries the matrix work (the k-loop), not the tile loop
_, lo, hi = min(cands)
c = collections.Counter()
for l in body[lo:hi + 1]:
    t = l.strip().split()
    if not t or t[0].startswith((";", ".")) or t[0].endswith(":"):
        continue
    op = t[0]
    if "mfma" in op:
        c["mfma"] += 1
    elif op.startswith("v_mov") or op.startswith("v_accvgpr"):
        c["v_mov/accvgpr"] += 1
    elif op.startswith("v_"):
        c["valu_other"] += 1
        c["  " + op] += 1
    elif op.startswith("ds_"):
        c[op] += 1
    elif op.startswith(("buffer_", "global_")):
        c["vmem " + op] += 1
    elif op.startswith("s_waitcnt"):
        c["s_waitcnt"] += 1
    elif op.startswith("s_barrier"):
        c["s_barrier"] += 1
    elif op.startswith("s_"):
        c["salu/other " + op.split("_")[1]] += 1
print(f"loop lines {lo}-{hi} of {sym}")
for k, v in sorted(c.items(), key=lambda kv: -kv[1]):
    print(f"  {v:5d}  {k}")
