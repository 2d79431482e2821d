#!/usr/bin/env python3
"""Summary of bench.py lines under gpurun_out/ (or given files): one row per
line -- ms per step, reads/s, NW busy, rounds, NW per read, seed ms, lanes."""
import glob
import json
import sys

files = sys.argv[1:] or sorted(glob.glob("gpurun_out/*.json"))
for f in files:
    if f.endswith(".last_call.json"):
        continue
    try:
        d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    except Exception:
        continue
    if "value" not in d:
        continue
    det, r = d.get("detail", {}), d.get("roofline", {})
    print("%-70s %9.3f ms %11.1f r/s busy %8.3f rnd %s nw/r %.4f seed %s cand %s" % (
        f.split("/")[-1][:70], d["ms_per_step"], d["value"], r.get("nw_busy_ms_per_step", 0), det.get("rounds"),
        det.get("nw_per_read", 0), det.get("ms_seed"), det.get("nw_launch_cand")))
