#!/usr/bin/env python3
"""Summarise the PMC passes of scripts/gpu_r2.sh (step `pmc`) into profiles/.

    python scripts/pmc_r2.py TAG

Passes (one counter group each, over one bench step --steps 1 --warmup 0):
  p1  SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES
  p2  FETCH_SIZE      p3  WRITE_SIZE      p4  GRBM_GUI_ACTIVE
Writes
  profiles/TAG_pmc.json     per kernel: launches and each counter's sum
  profiles/nw_traffic.json  HBM bytes per NW launch (bench.py roofline.traffic)
  profiles/nw_valu.json     VALU lane-instructions per DP cell of the NW kernel
                            (bench.py roofline.valu)
Counter handling follows /opt/skills/guides/MI355X_MICROARCH.md (HBM
section): FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half
the bytes of wide coalesced reads, so it is doubled; SQ cycle counters are
quad-cycles.  SQ_INSTS_VALU counts wave instructions (64 lanes)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(d):
    """{kernel: {"launches": n, counter: sum}} of one pass directory."""
    out = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for path in files:
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row["Kernel_Name"]
                out[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    for k in out:
        out[k]["launches"] = len(disp[k])
    return out


def main():
    tag = sys.argv[1]
    src = os.path.join(REPO, "gpurun_out")
    kern = defaultdict(dict)
    bench = None
    for i in range(1, 5):
        for k, v in counters(os.path.join(src, f"pmc_{tag}_p{i}")).items():
            kern[k].update(v)
        bj = os.path.join(src, f"pmc_{tag}_p{i}.json")
        if bench is None and os.path.exists(bj) and os.path.getsize(bj):
            bench = json.loads(open(bj).read().strip().splitlines()[-1])
    res = {k: dict(v) for k, v in kern.items()}
    prof = os.path.join(REPO, "profiles")
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as f:
        json.dump({"tag": tag, "note": "one bench step (--steps 1 --warmup 0), rocprofv3 --pmc, one counter group "
                   "per pass; FETCH_SIZE/WRITE_SIZE in KiB as reported (HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE, "
                   "MI355X_MICROARCH.md gfx950); SQ cycle counters in quad-cycles", "kernels": res}, f, indent=1)
    nwk = next((k for k in res if k.startswith("nw16_kernel")), None) or next(
        (k for k in res if k.startswith("nwp_kernel")), None) or next(
        (k for k in res if k.startswith("nwl_kernel")), None) or next(
        (k for k in res if k.startswith("nw_kernel")), None)
    if not nwk:
        print("no NW kernel in the passes")
        return
    v = res[nwk]
    n = max(int(v.get("launches", 1)), 1)
    kname = nwk.split("<")[0].split("(")[0]
    cfg = (bench or {}).get("config", {})
    wl = cfg.get("workload", "")
    config = next((c for c, p in (("c5w", "C5w:"), ("c5", "C5:"), ("c3", "C3 "), ("c2", "C2:")) if wl.startswith(p)),
                  "other")
    sfx = "" if config == "c2" else "_" + config      # bench.py: profiles/nw_{traffic,valu}[_CONFIG].json
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        fetch2, write = 2 * v["FETCH_SIZE"] * 1024, v["WRITE_SIZE"] * 1024
        cells = (bench or {}).get("detail", {}).get("nw_cells")
        with open(os.path.join(prof, f"nw_traffic{sfx}.json"), "w") as f:
            json.dump({"tag": tag, "kernel": kname, "config": config, "launches": n,
                       "hbm_bytes_per_launch": round((fetch2 + write) / n),
                       # per DP cell: bench.py scales it by the cells of ITS launches
                       # (launch sizes change with the lane count)
                       "nw_cells": cells,
                       "hbm_bytes_per_cell": round((fetch2 + write) / cells, 5) if cells else None,
                       "fetch_bytes_x2_per_launch": round(fetch2 / n), "write_bytes_per_launch": round(write / n),
                       "note": "one bench step (--steps 1 --warmup 0); FETCH_SIZE doubled per MI355X_MICROARCH.md "
                               "gfx950; KiB -> bytes"}, f, indent=1)
    if "SQ_INSTS_VALU" in v and bench:
        cells = bench["detail"]["nw_cells"]
        ipc = v["SQ_INSTS_VALU"] * 64.0 / cells
        with open(os.path.join(prof, f"nw_valu{sfx}.json"), "w") as f:
            json.dump({"tag": tag, "kernel": kname, "config": config, "launches": n,
                       "sq_insts_valu": v["SQ_INSTS_VALU"], "nw_cells": cells,
                       "lane_instr_per_cell": round(ipc, 4),
                       "valu_active_per_wave_cycle": round(v.get("SQ_ACTIVE_INST_VALU", 0) /
                                                           max(v.get("SQ_WAVE_CYCLES", 1), 1), 4),
                       "note": "SQ_INSTS_VALU (wave instructions) x 64 lanes / DP cells of the same step "
                               "(bench detail.nw_cells); one bench step"}, f, indent=1)
    for k, c in sorted(res.items()):
        print(k, {kk: round(vv, 1) for kk, vv in c.items()})


if __name__ == "__main__":
    main()
