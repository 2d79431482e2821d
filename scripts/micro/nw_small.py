#!/usr/bin/env python3
"""Latency of SMALL NW launches (the last rounds of a shard: ~1.4-2k
candidates per lane at the 1/8 shard, ~300 at C2's fourth round).

imsame_dev_nw_pairs on N pairs of a 2000-bp record vs a 150-bp read, per NW
form, kernel time from the library's own events (median of --reps).  Two read
kinds: "sim" (a window of the record, 1 % substitutions: a short diagonal
walk) and "rand" (an unrelated read: the rejected NWs of random reads, whose
paths wander).  With IMSAME_NW_PROF=1 the packed forms also print their phase
split on stderr.

    python scripts/micro/nw_small.py [--sizes 16,256,1400] [--out FILE]
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

FORMS = {                      # name -> (flags, environment)
    "int32": ("NW32", {}),
    "k19": ("NW16", {}),
    "k10": ("NW16", {"IMSAME_NW_K19": "0"}),
    "k5": ("NW16", {"IMSAME_NW_K": "5"}),
    "k3": ("NW16", {"IMSAME_NW_K": "3"}),
}


def pairs(n, kind, xlen, ylen, seed):
    import numpy as np
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    X = [acgt[rng.integers(0, 4, xlen)].tobytes() for _ in range(n)]
    Y = []
    for x in X:
        if kind == "rand":
            Y.append(acgt[rng.integers(0, 4, ylen)].tobytes())
            continue
        o = int(rng.integers(0, xlen - ylen))
        y = bytearray(x[o:o + ylen])
        for k in np.flatnonzero(rng.random(ylen) < 0.01):
            y[k] = acgt[(int("ACGT".index(chr(y[k]))) + 1) % 4]
        Y.append(bytes(y))
    return X, Y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,16,128,512,1400,4096")
    ap.add_argument("--forms", default="int32,k19,k10,k5,k3")
    ap.add_argument("--xlen", type=int, default=2000)
    ap.add_argument("--ylen", type=int, default=150)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import imsame_amd
    rows = []
    with imsame_amd.Device(0) as d:
        for kind in ("sim", "rand"):
            for n in [int(s) for s in a.sizes.split(",")]:
                X, Y = pairs(n, kind, a.xlen, a.ylen, 11 + n)
                ref = None
                for form in a.forms.split(","):
                    flag, env = FORMS[form]
                    saved = {k: os.environ.get(k) for k in env}
                    os.environ.update(env)
                    try:
                        p = d.params()
                        p.flags |= getattr(imsame_amd, "FLAG_" + flag)
                        ms = []
                        for _ in range(a.reps):
                            res, _, kms = d.nw_pairs(X, Y, params=p)
                            ms.append(kms)
                        key = [tuple(int(r[f]) for f in ("score", "bx", "by", "length", "identities")) for r in res]
                        if ref is None:
                            ref = key
                        same = key == ref
                    finally:
                        for k, v in saved.items():
                            if v is None:
                                os.environ.pop(k, None)
                            else:
                                os.environ[k] = v
                    row = {"kind": kind, "n": n, "form": form, "kernel_ms": round(statistics.median(ms), 4),
                           "min_ms": round(min(ms), 4), "same_as_first_form": same}
                    rows.append(row)
                    print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"xlen": a.xlen, "ylen": a.ylen, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
