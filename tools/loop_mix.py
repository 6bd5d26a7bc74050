#!/usr/bin/env python3
"""Instruction mix of the loops of one kernel in an llvm-objdump listing:
for each backward branch, the body's instruction count per class.
usage: loop_mix.py <listing.s> <kernel-name-substring> [min_body]"""
import collections
import re
import sys

path, name = sys.argv[1], sys.argv[2]
min_body = int(sys.argv[3]) if len(sys.argv) > 3 else 200
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if name in l and l.endswith(">:"))
end = next((i for i in range(start + 1, len(lines)) if re.match(r"^[0-9a-f]+ <.*>:$", lines[i])), len(lines))
ins = []
for l in lines[start + 1:end]:
    m = re.match(r"\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-F]+):", l)
    if m:
        ins.append((int(m.group(3), 16), m.group(1), m.group(2)))
base = ins[0][0]
idx = {a: i for i, (a, _, _) in enumerate(ins)}


def cls(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("ds_",)):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


for i, (a, op, args) in enumerate(ins):
    if not (op.startswith("s_cbranch") or op == "s_branch"):
        continue
    m = re.search(r"\+0x([0-9a-f]+)>", args)
    if not m:
        continue
    tgt = base + int(m.group(1), 16)
    j = idx.get(tgt)
    if j is None or j > i or i - j < min_body:
        continue
    body = ins[j:i + 1]
    c = collections.Counter(cls(o) for _, o, _ in body)
    v = collections.Counter(o for _, o, _ in body if o.startswith("v_"))
    print(f"loop {hex(tgt - base)}..{hex(a - base)}: {len(body)} instructions {dict(c)}")
    for o, k in v.most_common(18):
        print(f"   {o:28s} {k}")
