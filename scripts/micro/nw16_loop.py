#!/usr/bin/env python3
"""Measured issue ceiling of nw16_kernel's first-sweep loop.

Runs the packed NW kernel alone on the chip (imsame_dev_nw_pairs: one
persistent launch, every resident wave slot busy) over 150-bp reads against
2000-bp records (C2's shape; the column form the library picks for it), with
IMSAME_NW_PROF=1: the kernel sums each wave's s_memtime cycles (shader
cycles) per phase (nw16_kernel.hip `mark`).  From the first-sweep cycles:

  cycles per 2-step iteration of one wave = sweep1 / (tasks x (xlen+G-1)/2)
  SIMD issue rate = waves/SIMD x VALU per iteration / cycles per iteration

VALU per iteration is the ISA count of the fast loop (scripts/isa_blocks.py on
the built kernel; passed with --valu).  The ratio of that rate to the 2-cycle
peak (0.5 wave-instructions per SIMD cycle) is this loop's ceiling: what the
whole kernel could reach if every step were a fast first-sweep step with the
chip full and nothing else running.

    python scripts/micro/nw16_loop.py --valu 641 [--pairs 65536] [--out FILE]
    (641: the 19-column form's loop; 351: the 10-column form's, IMSAME_NW_K19=0)
"""
import argparse
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(a):
    sys.path.insert(0, REPO)
    import numpy as np
    import imsame_amd
    rng = np.random.default_rng(5)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    X = [acgt[rng.integers(0, 4, a.xlen)].tobytes() for _ in range(a.pairs)]
    # reads: a window of the record with 1 % substitutions (paths like C2's)
    Y = []
    for x in X:
        o = int(rng.integers(0, a.xlen - a.ylen))
        y = bytearray(x[o:o + a.ylen])
        for k in np.flatnonzero(rng.random(a.ylen) < 0.01):
            y[k] = acgt[(int("ACGT".index(chr(y[k]))) + 1) % 4]
        Y.append(bytes(y))
    with imsame_amd.Device(0) as d:
        p = d.params()
        p.flags |= imsame_amd.FLAG_NW16
        for _ in range(a.reps):
            d.nw_pairs(X, Y, params=p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--valu", type=float, required=True, help="VALU instructions per fast-loop iteration (2 steps)")
    ap.add_argument("--pairs", type=int, default=65536)
    ap.add_argument("--xlen", type=int, default=2000)      # C2's records (LDS: 4 blocks of 4 waves per CU)
    ap.add_argument("--ylen", type=int, default=150)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--waves-per-simd", type=float, default=None,
                    help="resident waves per SIMD (default: the launch's blocks x 4 waves / 1024 SIMDs)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a)
    env = dict(os.environ, IMSAME_NW_PROF="1")
    p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"] + sys.argv[1:], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=900)
    err = p.stderr.decode(errors="replace")
    if p.returncode:
        sys.exit(err[-2000:])
    runs = []
    for m in re.finditer(r"\[nwprof-raw\] (.*)", err):
        f = m.group(1).split()
        runs.append({f[k]: float(f[k + 1]) for k in range(0, len(f) - 1, 2)})
    r = runs[-1]                              # warm
    G, GPW = int(r["G"]), int(r["GPW"])
    tasks = -(-int(r["cand"]) // (2 * GPW))
    iters = (a.xlen + G - 1) / 2.0
    tot = sum(r[k] for k in ("setup", "sweep1", "reduce", "sweep2", "walk"))
    cyc_iter = r["sweep1"] / (tasks * iters)
    if a.waves_per_simd is None:                           # persistent launch: blocks x 4 waves over 1024 SIMDs
        a.waves_per_simd = min(r["blocks"] * 4, tasks) / 1024.0
    rate = a.waves_per_simd * a.valu / cyc_iter           # wave-instructions per SIMD cycle
    tot_cyc = sum(r[k] for k in ("setup", "sweep1", "reduce", "sweep2", "walk"))
    # shader clock: the waves' s_memtime cycles over their s_memrealtime ticks
    # (100 MHz), MI355X_MICROARCH.md's in-kernel clock (round 4 divided by the
    # launch's duration x its waves, which assumed every wave ran the whole
    # launch: 1.94 GHz, too low)
    ghz = tot_cyc / r["rt"] * 0.1 if r.get("rt") else None
    out = {"kernel": "nw16_kernel", "form": int(r["k"]), "what": "first-sweep fast loop, chip full, kernel alone",
           "pairs": int(r["cand"]), "xlen": a.xlen, "ylen": a.ylen, "G": G, "GPW": GPW, "tasks": tasks,
           "valu_per_iteration": a.valu, "waves_per_simd": a.waves_per_simd,
           "cycles_per_iteration_per_wave": round(cyc_iter, 1),
           "cycles_per_valu_per_simd": round(cyc_iter / (a.waves_per_simd * a.valu), 3),
           "simd_valu_rate": round(rate, 4), "mix_ceiling_frac": round(rate / 0.5, 4),
           "sweep1_share": round(r["sweep1"] / tot, 4), "kernel_ms": r["ms"],
           "shader_clock_ghz": round(ghz, 3) if ghz else None,
           # not comparable with the bench's cells/s: the micro's candidates
           # carry no predicted window, so every one takes a second sweep
           "micro_cells_per_s_no_windows": round(a.pairs * a.xlen * a.ylen / (r["ms"] / 1e3), 1),
           "raw": runs}
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
