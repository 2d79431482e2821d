#!/usr/bin/env python3
"""Basic blocks of one kernel in a hipcc -S listing, with VALU/VMEM/SALU
counts and back-edges (loops): python scripts/isa_blocks.py file.s SYMBOL"""
import re
import sys
from collections import Counter

path, sym = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur, name = [], [], "entry"
for l in lines[start + 1:end]:
    m = re.match(r"^(\.LBB[0-9_]+):", l)
    if m:
        blocks.append((name, cur)); name, cur = m.group(1), []
        continue
    s = l.strip()
    if not s or s.startswith(";") or s.startswith("."):
        continue
    cur.append(s.split(";")[0].strip())
blocks.append((name, cur))
order = {n: k for k, (n, _) in enumerate(blocks)}
for k, (n, ins) in enumerate(blocks):
    c = Counter()
    for i in ins:
        op = i.split()[0]
        c["valu" if op.startswith("v_") else "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_"))
          else "lds" if op.startswith("ds_") else "salu" if op.startswith("s_") else "other"] += 1
    tgt = [re.search(r"(\.LBB[0-9_]+)", i).group(1) for i in ins if i.startswith("s_cbranch") or i.startswith("s_branch")]
    back = [t for t in tgt if t in order and order[t] <= k]
    if len(ins) > 40 or back:
        print(f"{n:14s} n={len(ins):5d} valu={c['valu']:5d} vmem={c['vmem']:3d} lds={c['lds']:3d} salu={c['salu']:3d}"
              f" back->{back}")
if len(sys.argv) > 3:
    want = sys.argv[3]
    for n, ins in blocks:
        if n == want:
            ops = Counter(i.split()[0] for i in ins)
            for op, k in ops.most_common():
                print(f"  {op:28s} {k}")
