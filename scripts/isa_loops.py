#!/usr/bin/env python3
"""Innermost loops of one kernel in a hipcc -S listing: per loop (header
label), its VALU / scratch (spill) / vmem instruction counts, from the
'Loop Header: Depth=N' / 'in Loop: Header=' annotations LLVM writes:
python scripts/isa_loops.py file.s SYMBOL [min_depth]"""
import re
import sys
from collections import defaultdict

path, sym = sys.argv[1], sys.argv[2]
mind = int(sys.argv[3]) if len(sys.argv) > 3 else 2
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
cur, depth = None, 0
stat = defaultdict(lambda: defaultdict(int))
for l in lines[start + 1:end]:
    m = re.match(r"^(\.LBB[0-9_]+|; %bb\.[0-9]+):.*?(?:Loop Header: Depth=(\d+)|Header=BB([0-9_]+) Depth=(\d+))?\s*$", l)
    if m:
        if m.group(2):
            cur, depth = "BB" + m.group(1)[4:], int(m.group(2))
        elif m.group(3):
            cur, depth = "BB" + m.group(3), int(m.group(4))
        elif m.group(1).startswith(".LBB"):
            cur, depth = None, 0
        continue
    s = l.strip()
    if not s or s.startswith((";", ".")) or cur is None or depth < mind:
        continue
    op = s.split()[0]
    st = stat[(cur, depth)]
    st["n"] += 1
    if op.startswith("v_"): st["valu"] += 1
    if op.startswith("scratch_"): st["scratch"] += 1
    if op.startswith(("global_", "buffer_")): st["vmem"] += 1
    if op.startswith("ds_"): st["lds"] += 1
for (h, d), st in stat.items():
    print(f"{h:12s} depth={d} n={st['n']:5d} valu={st['valu']:5d} scratch={st['scratch']:3d} vmem={st['vmem']:3d} lds={st['lds']:3d}")
