#!/usr/bin/env python3
"""Golden vectors for the all-vs-all metagenome path,
produced by the REFERENCE compiled from its own sources (oracle/_ref/IMSAME,
oracle/_ref/revComp; oracle/Makefile `ref`).

The reference's driver, bin/all_vs_all_metagenomes_IMSAME.sh, is a bash loop
around those two programs.  Its prebuilt bin/IMSAME is never run, so this
script replays the loop (all_vs_all_metagenomes_IMSAME.sh:21-56: ls order,
pairs i < j, X-Y.align then revComp Y -> Y.r.EXT and X-Y.r.align) with the
compiled binaries, in a scratch directory, and freezes the outputs.

    python tests/golden/make_avav_golden.py

Fixture (data only): tests/golden/avav/
  in/<name>.fa          three synthetic metagenomes (shared genome pool,
                        distinct abundances, both strands; one file 60-column
                        CRLF with N runs and lower case -- revComp drops the
                        CR, so its reverse-complement database has k-mers the
                        forward one lacks)
  expected.json         per THR: run list, exit codes, [INFO] summary lines,
                        record multisets (THR > 1)
  T1/<X-Y[.r]>.align.gz .align bytes for THR = 1 (file order is defined)
"""
import gzip
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref")
OUT = os.path.join(HERE, "avav")
sys.path.insert(0, REPO)
from tests import synth  # noqa: E402
from tests.golden_io import info_lines, err_lines, record_multisets  # noqa: E402

COV, SIM, EXT = "0.5", "0.5", "fa"
THREADS = [1, 3]


def crlf_fasta(seq, starts, prefix, width, rng):
    b = bytearray(seq.tobytes())
    # N runs (database k-mer breaks) and lower case (kept by both loaders)
    for p in rng.integers(0, len(b), len(b) // 400):
        b[p] = ord("N")
    for p in rng.integers(0, len(b), len(b) // 50):
        b[p] = b[p] | 0x20 if b[p] != ord("N") else b[p]
    ends = list(starts[1:].tolist()) + [len(b)]
    out = []
    for i, (s, e) in enumerate(zip(starts.tolist(), ends)):
        out.append(f">{prefix}_{i} sample\r\n".encode())
        for k in range(s, e, width):
            out.append(bytes(b[k:min(e, k + width)]) + b"\r\n")
    return b"".join(out)


def make_inputs(d):
    pool = synth.make_genome_pool(3, 12_000, seed=61)
    specs = [("mgA", [0.6, 0.3, 0.1], 0), ("mgB", [0.2, 0.3, 0.5], 80), ("mgC", [0.3, 0.4, 0.3], -60)]
    for k, (name, ab, width) in enumerate(specs):
        seq, st = synth.make_metagenome_arr(pool, ab, 300, 150, seed=62 + k)
        if width < 0:
            blob = crlf_fasta(seq, st, name, -width, np.random.default_rng(70 + k))
        else:
            blob = synth.to_fasta(seq, st, name, width=width)
        open(os.path.join(d, f"{name}.{EXT}"), "wb").write(blob)


def replay_script(mdir, odir, thr):
    """all_vs_all_metagenomes_IMSAME.sh:21-56 with the compiled reference."""
    names = sorted(f[:-len(EXT) - 1] for f in os.listdir(mdir) if f.endswith("." + EXT))
    runs = []
    for i in range(len(names)):
        for j in range(i, len(names)):
            if i == j:
                continue
            X, Y = names[i], names[j]
            for rev in (0, 1):
                tag = f"{X}-{Y}{'.r' if rev else ''}"
                db = os.path.join(mdir, f"{Y}.{EXT}")
                if rev:
                    db = os.path.join(mdir, f"{Y}.r.{EXT}")
                    subprocess.run([os.path.join(REF, "revComp"), os.path.join(mdir, f"{Y}.{EXT}"), db], check=True)
                p = subprocess.run([os.path.join(REF, "IMSAME"), "-query", os.path.join(mdir, f"{X}.{EXT}"),
                                    "-db", db, "-n_threads", str(thr), "-coverage", COV, "-identity", SIM,
                                    "-out", os.path.join(odir, tag + ".align")],
                                   stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
                if rev:
                    os.remove(db)
                runs.append(dict(tag=tag, rc=p.returncode, info=info_lines(p.stdout), err=err_lines(p.stdout)))
    return runs


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    shutil.rmtree(OUT, ignore_errors=True)
    os.makedirs(os.path.join(OUT, "in"))
    os.makedirs(os.path.join(OUT, "T1"))
    make_inputs(os.path.join(OUT, "in"))
    meta = {"cov": COV, "sim": SIM, "ext": EXT, "threads": {}}
    for thr in THREADS:
        with tempfile.TemporaryDirectory() as td:
            mdir, odir = os.path.join(td, "m"), os.path.join(td, "o")
            shutil.copytree(os.path.join(OUT, "in"), mdir)
            os.makedirs(odir)
            runs = replay_script(mdir, odir, thr)
            for r in runs:
                blob = open(os.path.join(odir, r["tag"] + ".align"), "rb").read()
                if thr == 1:
                    with open(os.path.join(OUT, "T1", r["tag"] + ".align.gz"), "wb") as f:
                        f.write(gzip.compress(blob, mtime=0))
                else:
                    r["headers"], r["body_sha1s"] = record_multisets(blob)
                print(thr, r["tag"], r["rc"], r["info"][:1], len(blob))
            meta["threads"][str(thr)] = runs
    json.dump(meta, open(os.path.join(OUT, "expected.json"), "w"), indent=0)


if __name__ == "__main__":
    main()
