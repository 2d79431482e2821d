#!/usr/bin/env python3
"""NW launches of a rocprofv3 kernel trace: count, mean duration and the
union of their intervals (the time the device ran NW, which with two lanes
is less than count x mean) -- the check of bench.py's roofline
(`avg_launch_ms`, `nw_busy_ms`) against the profiler.

    python scripts/nw_busy.py gpurun_out/prof_TAG/kt_kernel_trace.csv [--kernel nw16_kernel] [--last K]
--last K: only the last K launches (the timed steps of `bench.py --steps S
--warmup W`: K = S x launches per step)."""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="nw16_kernel")
    ap.add_argument("--last", type=int, default=0)
    a = ap.parse_args()
    iv = []
    with open(a.trace) as f:
        for row in csv.DictReader(f):
            if row["Kernel_Name"].startswith(a.kernel):
                iv.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    iv.sort()
    if a.last:
        iv = iv[-a.last:]
    busy, lo, hi = 0, None, None
    for s, e in iv:
        if hi is None or s > hi:
            if hi is not None:
                busy += hi - lo
            lo, hi = s, e
        else:
            hi = max(hi, e)
    if hi is not None:
        busy += hi - lo
    tot = sum(e - s for s, e in iv)
    print(f"{a.kernel}: {len(iv)} launches, mean {tot / max(len(iv), 1) / 1e6:.3f} ms, "
          f"sum {tot / 1e6:.3f} ms, union (busy) {busy / 1e6:.3f} ms, overlap {tot / max(busy, 1):.3f}")


if __name__ == "__main__":
    main()
