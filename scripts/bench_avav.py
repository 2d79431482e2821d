#!/usr/bin/env python3
"""Benchmark of the all-vs-all metagenome job (BASELINE.json configs[3],
SURVEY.md 8(d) C4): 4 synthetic metagenomes x R reads x 150 bp drawn from a
shared pool of 10 x 5 Mbp genomes with distinct abundance vectors (seeds
44-47), all 12 runs (6 pairs x forward / reverse complement) of
bin/all_vs_all_metagenomes_IMSAME.sh as ONE imsame_all_vs_all job.

    python scripts/bench_avav.py [--reads 2000000] [--threads 16] [--devices N] [--text]

Without --text the outpath does not exist, so -- exactly as the stock IMSAME
whose fopen of -out fails -- no .align text is written and the job time is
parse + revComp + index + alignment; with --text the .align files are
written under $TMPDIR (large: ~1 KB per accepted read).
Prints one JSON line: read alignments per second over the whole job and the
driver's per-run breakdown.
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tests import synth  # noqa: E402

AVAV = os.path.join(REPO, "imsame_amd", "bin", "imsame_all_vs_all")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--genomes", type=int, default=10)
    ap.add_argument("--genome-bp", type=int, default=5_000_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--devices", default=None)
    ap.add_argument("--text", action="store_true")
    a = ap.parse_args()
    td = tempfile.mkdtemp(prefix="avav_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        mdir = os.path.join(td, "m")
        os.makedirs(mdir)
        t0 = time.time()
        pool = synth.make_genome_pool(a.genomes, a.genome_bp, seed=44)
        import numpy as np
        for k in range(4):
            ab = np.random.default_rng(100 + k).dirichlet(np.ones(a.genomes))
            seq, st = synth.make_metagenome_arr(pool, ab, a.reads, 150, seed=44 + k)
            synth.write_fasta(os.path.join(mdir, f"mg{k}.fasta"), seq, st, f"mg{k}", width=0)
        t_gen = time.time() - t0
        odir = os.path.join(td, "o" if a.text else "missing")
        if a.text:
            os.makedirs(odir)
        cmd = [AVAV, mdir, "0.5", "0.5", str(a.threads), "fasta", odir]
        if a.devices:
            cmd += ["-devices", a.devices]
        t0 = time.perf_counter()
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
        wall = time.perf_counter() - t0
        if p.returncode:
            sys.stderr.write(p.stderr.decode()[-3000:])
            raise SystemExit(p.returncode)
        err = p.stderr.decode()
        runs = [dict(zip(("out", "reads", "accepted", "nw", "cells", "shards", "align_ms"),
                         (m[0], int(m[1]), int(m[2]), int(m[3]), int(m[4]), int(m[5]), float(m[6]))))
                for m in re.findall(r"\] (\S+): reads=(\d+) accepted=(\d+) nw=(\d+) cells=(\d+) shards=(\d+) "
                                    r"(?:batches=\d+ )?align_ms\(max\)=([\d.]+)", err)]
        if not runs:
            sys.stderr.write(err[-3000:])
            raise SystemExit("no per-run lines in the driver's output")
        job = re.search(r"(\d+) runs, (\d+) skipped, (\d+) device contexts, ([\d.]+) s", err)
        total_reads = sum(r["reads"] for r in runs)
        align_s = sum(r["align_ms"] for r in runs) / 1e3
        pl = re.search(r"\[imsame_all_vs_all\] phase (.*)", err)
        phases = dict(re.findall(r"(\w+)=([\d.]+)", pl.group(1))) if pl else {}
        line = {"metric": "read alignments/sec, all-vs-all metagenomes (4 x %d reads, 12 runs)" % a.reads,
                "value": round(total_reads / wall, 1), "unit": "reads/s", "wall_s": round(wall, 3),
                "align_s_sum": round(align_s, 3), "align_only_reads_per_s": round(total_reads / align_s, 1),
                "runs": len(runs), "devices": int(job.group(3)) if job else None, "text": a.text,
                "gen_s": round(t_gen, 1), "phases_s": {k: float(v) for k, v in phases.items()},
                "accepted_per_run": [r["accepted"] for r in runs],
                "nw_per_read": round(sum(r["nw"] for r in runs) / max(total_reads, 1), 4),
                "config": {"workload": "C4: all_vs_all_metagenomes_IMSAME.sh path, 4 synthetic metagenomes "
                                       "(pool %d x %d bp), BASELINE.json configs[3]" % (a.genomes, a.genome_bp),
                           "n_threads_semantic": a.threads}}
        print(json.dumps(line), flush=True)
    finally:
        shutil.rmtree(td, ignore_errors=True)


if __name__ == "__main__":
    main()
