#!/usr/bin/env python3
"""Summarise the rocprofv3 outputs of scripts/gpu_profile.sh into profiles/.

    python scripts/pmc_summary.py TAG [--out profiles]

Reads gpurun_out/prof_TAG/kt_kernel_stats.csv (kernel trace --stats) and the
two PMC passes gpurun_out/pmc_{fetch,write}_TAG/pmc_counter_collection.csv,
and writes
    profiles/TAG_kernel_stats.csv      (copy of the rocprofv3 --stats summary)
    profiles/TAG_pmc.json              (per-kernel launches, avg FETCH/WRITE bytes)
    profiles/nw_traffic.json           (HBM bytes per nw_kernel launch, read by bench.py)

Counter handling follows /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of wide coalesced reads, so it is doubled (an upper bound for the
narrower accesses this path also makes; the guide calls other widths
uncalibrated); WRITE_SIZE is taken as is (the NW traceback is one dword per
lane, 256-B wave stores).
"""
import argparse
import csv
import json
import os
import shutil
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    acc = defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            a = acc[row["Kernel_Name"]]
            a[0] += 1
            a[1] += float(row["Counter_Value"]) * 1024.0
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--src", default=os.path.join(REPO, "gpurun_out"))
    ap.add_argument("--out", default=os.path.join(REPO, "profiles"))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    stats = os.path.join(a.src, f"prof_{a.tag}", "kt_kernel_stats.csv")
    shutil.copy(stats, os.path.join(a.out, f"{a.tag}_kernel_stats.csv"))
    fetch = per_kernel(os.path.join(a.src, f"pmc_fetch_{a.tag}", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(a.src, f"pmc_write_{a.tag}", "pmc_counter_collection.csv"), "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        nf, bf = fetch.get(k, [0, 0.0])
        nw, bw = write.get(k, [0, 0.0])
        n = max(nf, nw, 1)
        out[k] = {"launches": n, "fetch_bytes_raw": bf, "fetch_bytes_x2": 2 * bf, "write_bytes": bw,
                  "hbm_bytes_per_launch": (2 * bf + bw) / n}
    with open(os.path.join(a.out, f"{a.tag}_pmc.json"), "w") as f:
        json.dump({"tag": a.tag, "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md gfx950 correction; "
                   "KiB -> bytes; one bench step (--steps 1 --warmup 0)", "kernels": out}, f, indent=1)
    kname = "nw16_kernel" if "nw16_kernel" in out else "nw_kernel"      # the NW kernel the bench ran
    nw = out.get(kname)
    if nw:
        with open(os.path.join(a.out, "nw_traffic.json"), "w") as f:
            json.dump({"tag": a.tag, "kernel": kname, "launches": nw["launches"],
                       "hbm_bytes_per_launch": round(nw["hbm_bytes_per_launch"]),
                       "fetch_bytes_x2_per_launch": round(nw["fetch_bytes_x2"] / nw["launches"]),
                       "write_bytes_per_launch": round(nw["write_bytes"] / nw["launches"]),
                       "note": "one bench step (--steps 1 --warmup 0); FETCH_SIZE doubled per "
                               "MI355X_MICROARCH.md gfx950; KiB -> bytes"}, f, indent=1)
    for k, v in out.items():
        print(f"{k:40s} n={v['launches']:5d}  fetch(x2)={v['fetch_bytes_x2']/1e9:9.3f} GB  "
              f"write={v['write_bytes']/1e9:9.3f} GB")


if __name__ == "__main__":
    main()
