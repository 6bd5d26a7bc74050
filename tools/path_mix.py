#!/usr/bin/env python3
"""Instruction mix along the fall-through path of a kernel's loop in an
llvm-objdump listing: from address FROM, conditional branches not taken
(the rare paths), unconditional branches followed, until address TO.
usage: path_mix.py <listing.s> <kernel-substring> <from-hex> <to-hex>"""
import collections
import re
import sys

path, name, a0, a1 = sys.argv[1], sys.argv[2], int(sys.argv[3], 16), int(sys.argv[4], 16)
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if name in l and l.endswith(">:"))
ins, base = [], None
for l in lines[start + 1:]:
    if re.match(r"^[0-9a-f]+ <.*>:$", l):
        break
    m = re.match(r"\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-F]+):", l)
    if m:
        a = int(m.group(3), 16)
        base = a if base is None else base
        t = re.search(r"\+0x([0-9a-f]+)>", l)
        ins.append((a - base, m.group(1), m.group(2), int(t.group(1), 16) if t else None))
idx = {a: i for i, (a, _, _, _) in enumerate(ins)}
i = idx[a0]
seen = collections.Counter()
ops = collections.Counter()
steps = 0
while ins[i][0] != a1 and steps < 200000:
    a, op, args, t = ins[i]
    steps += 1
    ops[op] += 1
    if op == "s_branch" and t > a:  # (backward jumps: inner loops, taken once)
        i = idx[t]
        continue
    i += 1
cls = collections.Counter()
for op, k in ops.items():
    c = ("lds" if op.startswith("ds_") else "vmem" if op.startswith(("buffer_", "global_")) else
         "waitcnt" if op.startswith("s_waitcnt") else "salu" if op.startswith("s_") else
         "valu" if op.startswith("v_") else "other")
    cls[c] += k
print(f"{steps} instructions on the path: {dict(cls)}")
for op, k in ops.most_common(40):
    print(f"   {op:30s} {k}")
