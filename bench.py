#!/usr/bin/env python3
"""Benchmark of the IMSAME seed-and-extend hot path on MI355X.

Metric (BASELINE.json): reads aligned/sec (node), 1M x 150 bp synthetic
Illumina-like reads vs a 50 Mbp synthetic reference (configs[1]).

One step = one imsame_dev_align pass over the rank's 1M-read shard (seed
scan + ungapped/e-value + NW wavefront + backtrack + acceptance + D2H of the
per-read results), inputs resident in HBM.  N GPUs: one process per GPU
(torchrun), each aligns its OWN 1M-read shard against its replica of the
index (weak scaling, no data-path collective); the accepted-read counters are
all-reduced over RCCL at the end.  value = N * 1M * steps / max-over-ranks
wall time of the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "reads aligned/sec (node), 1M×150bp vs 50Mbp ref, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md, chip-level parameters


# BASELINE.json configs, per GPU (SURVEY 8(d) canonical inputs).  c2 is the
# metric's configuration and the default; c3 is configs[2]'s per-GPU shard
# (10M reads / 8 GPUs vs 500 Mbp); c5 is configs[4] (ONT-like 10 kbp reads,
# raised MAX_READ_SIZE, reads capped per GPU by --reads).
CONFIGS = {
    "c2": dict(reads=1_000_000, read_len=150, ref_bp=50_000_000, record_bp=2_000, ont=False, max_rs=None,
               cpu_sample=40_000, seeds=(42, 43),
               workload="C2: 1M x 150 bp Illumina-like reads per GPU vs 50 Mbp synthetic reference "
                        "(2 kbp records), BASELINE.json configs[1]"),
    "c3": dict(reads=1_250_000, read_len=150, ref_bp=500_000_000, record_bp=2_000, ont=False, max_rs=None,
               cpu_sample=4_000, seeds=(43, 44),
               workload="C3 per-GPU shard: 1.25M x 150 bp reads per GPU (10M over 8) vs 500 Mbp synthetic "
                        "reference (2 kbp records), BASELINE.json configs[2]"),
    "c5": dict(reads=100_000, read_len=10_000, ref_bp=50_000_000, record_bp=2_000, ont=True, max_rs=10_001,
               cpu_sample=0, seeds=(42, 48),
               workload="C5: 10 kbp ONT-like reads (5% sub, 2.5% ins, 2.5% del) vs 50 Mbp synthetic reference, "
                        "MAX_READ_SIZE raised to 10001, BASELINE.json configs[4]"),
}


def nw_kernel_name(read_len, record_bp, igap=-5, egap=-2):
    """The NW kernel imsame_dev.hip:plan_nw picks for this shape (mirror of
    nw16_kernel.hip:nw16_fits for the default gap parameters)."""
    if igap > 0 or egap > 0 or read_len > 160:
        return "nw_kernel"
    ycols = -(-read_len // 10) * 10
    R = 4 * ycols - igap - egap * (record_bp + 64 + ycols + 2) + 16
    return "nw16_kernel" if R <= 8191 else "nw_kernel"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2",
                    help="BASELINE.json workload (c2 = the metric's config; c3/c5 are stress runs)")
    ap.add_argument("--reads", type=int, default=None, help="reads per GPU (default: the config's)")
    ap.add_argument("--read-len", type=int, default=None)
    ap.add_argument("--ref-bp", type=int, default=None)
    ap.add_argument("--record-bp", type=int, default=None)
    ap.add_argument("--n-threads", type=int, default=16, help="reference -n_threads semantics")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="reads in the CPU baseline sample (0: skip; default: the config's)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-kind", choices=("auto", "port", "reference"), default="auto",
                    help="auto: the compiled reference (oracle/_ref/IMSAME) when present, else the port")
    ap.add_argument("--slice-bases", type=int, default=0,
                    help="search the database in slices of at most this many bases, one slice's index in HBM "
                         "at a time (imsame_dev_align_sliced; the index rebuilds are inside the timed step)")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "nw_traffic.json"))
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    for k in ("reads", "read_len", "ref_bp", "record_bp", "cpu_sample"):
        if getattr(a, k) is None:
            setattr(a, k, cfg[k])
    return a


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import imsame_amd
    from tests import synth

    # synthetic C2 inputs: the reference is replicated, each rank has its own reads
    cfg = CONFIGS[a.config]
    ref, rst = synth.make_reference_arr(a.ref_bp, a.record_bp, seed=cfg["seeds"][0])
    gen = synth.make_long_reads_arr if cfg["ont"] else synth.make_reads_arr
    q, qs = gen(ref, a.reads, a.read_len, seed=cfg["seeds"][1] + 1000 * rank)
    dev = imsame_amd.Device(local)
    t0 = time.time()
    dev.index(ref, rst)
    t_index = time.time() - t0
    dev.set_query(q, qs)                               # H2D once: inputs resident in HBM
    params = dev.params(max_read_size=cfg["max_rs"]) if cfg["max_rs"] else dev.params()

    n_slices = 1

    def step():
        nonlocal n_slices
        if a.slice_bases:
            res, paths, st, n_slices = dev.align_sliced(ref, rst, a.slice_bases, n_threads=a.n_threads,
                                                        params=params)
            return res, paths, st
        return dev.align(0, a.reads, n_threads=a.n_threads, params=params)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(a.warmup):
        step()
    barrier()
    stats = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res, _, st = step()
        stats.append(st.as_dict())
    barrier()
    elapsed = time.perf_counter() - t0
    accepted = int((res["status"] == 1).sum())
    if dist is not None:
        from imsame_amd.dist import all_reduce     # RCCL: max of the clocks, sum of the counters
        elapsed = all_reduce([elapsed], op="max")[0]
        accepted_all = int(all_reduce([accepted])[0])
    else:
        accepted_all = accepted
    total_reads = world * a.reads * a.steps
    value = total_reads / elapsed

    # dominant kernel: nw_kernel.  Algorithmic bytes per NW candidate (SURVEY
    # 8(d)): record + read + 2 B/cell traceback floor; HIP events on the
    # library's own stream bracket every NW launch.
    nw_ms = sum(s["ms_nw"] for s in stats)
    nw_launches = sum(s["nw_launches"] for s in stats)
    cells = sum(s["nw_cells"] for s in stats)
    n_nw = sum(s["n_nw"] for s in stats)
    seq_bytes = n_nw * (a.record_bp + a.read_len)
    alg_bytes = 2 * cells + seq_bytes
    achieved = alg_bytes / (nw_ms / 1e3) / 1e9 if nw_ms else 0.0
    kernel = nw_kernel_name(a.read_len, a.record_bp) if not stats[-1]["nw_launches"] or a.read_len <= 160 \
        else "nw_kernel"
    traffic = None
    if os.path.exists(a.traffic_json):
        try:
            tj = json.load(open(a.traffic_json))
            if tj.get("kernel") == kernel:          # PMC pass of THIS kernel (profiles/)
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": kernel, "launches": nw_launches,
                "avg_launch_ms": round(nw_ms / max(nw_launches, 1), 4),
                "alg_bytes_per_launch": int(alg_bytes / max(nw_launches, 1)),
                "cells_per_s": round(cells / (nw_ms / 1e3), 1) if nw_ms else 0.0}

    cpu = None
    if rank == 0 and world == 1 and a.cpu_sample > 0:
        if a.slice_bases:
            dev.index(ref, rst)                     # the sample is checked against the whole index
        cpu = cpu_baseline(dev, ref, rst, q, qs, a, params)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "reads/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int32", "data": "synthetic",
            "config": {"workload": cfg["workload"] + (f"; database searched in {n_slices} slices of <= "
                                                       f"{a.slice_bases} bases" if a.slice_bases else ""),
                       "reads_per_gpu": a.reads, "read_len": a.read_len, "ref_bp": a.ref_bp,
                       "record_bp": a.record_bp, "n_threads_semantic": a.n_threads,
                       "parallelism": f"dp{world} (read shards, replicated index)"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "detail": {"accepted_reads": accepted_all, "index_build_s": round(t_index, 3),
                       "rounds": stats[-1]["rounds"], "nw_per_read": round(stats[-1]["n_nw"] / a.reads, 4),
                       "hits_per_read": round(stats[-1]["n_hits"] / a.reads, 2),
                       "ms_seed": round(stats[-1]["ms_seed"], 3), "ms_nw": round(stats[-1]["ms_nw"], 3),
                       "ms_align_call": round(stats[-1]["ms_total"], 3)},
        }
        print(json.dumps(line), flush=True)
    dev.close()
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(dev, ref, rst, q, qs, a, params):
    """The oracle (clean-room CPU restatement, 'port') on the host cores, on a
    bounded sample: the first cpu_sample reads of the rank-0 shard taken as a
    query of their own, -n_threads cpu_threads, alignment phase only (index
    build excluded, as for the GPU).  The GPU then aligns the same sample view
    with the same -n_threads and every per-read result is compared."""
    from tests.oracle_bind import Oracle
    from imsame_amd import PARITY_FIELDS
    o = Oracle.load()
    n = min(a.cpu_sample, len(qs))
    qv = q[:int(qs[n])] if n < len(qs) else q
    po = o.params(max_read_size=params.max_read_size)
    rc, exp, _ = o.align(ref, rst, qv, qs[:n], po, a.cpu_threads)
    o.lib.or_last_align_seconds.restype = C.c_double
    secs = o.lib.or_last_align_seconds()
    dev.set_query(qv, qs[:n])
    got, _, _ = dev.align(0, n, n_threads=a.cpu_threads, params=params)
    same = int(np.all([exp[f] == got[f] for f in PARITY_FIELDS], axis=0).sum())
    port = {"value": round(n / secs, 1), "unit": "reads/s", "cores": a.cpu_threads, "kind": "port",
            "sample": f"first {n} reads of the rank-0 shard as their own query, oracle/imsame_oracle.c "
                      f"-n_threads {a.cpu_threads}, alignment-phase wall {secs:.2f} s",
            "sample_reads_identical_to_gpu": same, "sample_reads_compared": n}
    ref_bin = os.path.join(REPO, "oracle", "_ref", "IMSAME")
    if a.cpu_kind == "port" or (a.cpu_kind == "auto" and not os.access(ref_bin, os.X_OK)):
        return port
    r = run_reference(ref_bin, ref, rst, qv, qs[:n], a.cpu_threads)
    gpu_acc = int((got["status"] == 1).sum())
    return {"value": round(n / r["align_s"], 1), "unit": "reads/s", "cores": a.cpu_threads, "kind": "reference",
            "sample": f"first {n} reads of the rank-0 shard as their own query vs the same database, "
                      f"IMSAME compiled from the reference sources (oracle/Makefile ref, gcc -O3) -n_threads "
                      f"{a.cpu_threads}; alignment phase = process wall {r['wall_s']:.2f} s minus its single-threaded "
                      f"setup phases {r['setup_s']:.2f} s = {r['align_s']:.2f} s",
            "reference_accepted": r["accepted"], "gpu_accepted": gpu_acc,
            "port": port}


def run_reference(ref_bin, ref, rst, q, qs, threads):
    """Run the compiled reference on FASTA files of the sample (test
    infrastructure: the CPU baseline only).  Its timing lines use clock() --
    CPU time summed over threads -- so the alignment phase is the process's
    wall time minus its three single-threaded setup phases (quick table,
    database + hash table, query; IMSAME.c:102,295,407), for which clock()
    equals wall time.  Process start-up and the heap teardown
    after the last line stay in, so this slightly overstates the phase."""
    import re
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        dbf, qf = os.path.join(td, "db.fa"), os.path.join(td, "q.fa")
        b = ref.tobytes()
        ends = rst[1:].tolist() + [len(ref)]
        with open(dbf, "wb") as f:
            for i, (s0, s1) in enumerate(zip(rst.tolist(), ends)):
                rec = b[s0:s1]
                f.write(b">ref_%d\n" % i + b"\n".join(rec[j:j + 80] for j in range(0, len(rec), 80)) + b"\n")
        b = q.tobytes()
        qe = qs[1:].tolist() + [len(q)]
        with open(qf, "wb") as f:
            f.write(b"".join(b">read_%d\n" % i + b[s0:s1] + b"\n" for i, (s0, s1) in enumerate(zip(qs.tolist(), qe))))
        t0 = time.monotonic()
        p = subprocess.run([ref_bin, "-db", dbf, "-query", qf, "-n_threads", str(threads)],
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=600)
        wall = time.monotonic() - t0
    out = p.stdout.decode(errors="replace")
    setup = [float(x) for x in re.findall(r"(?:Initialization took|building took|Took) ([0-9.eE+-]+) seconds", out)]
    acc = re.search(r"\[INFO\] (\d+) reads \(", out)
    if p.returncode != 0 or len(setup) != 3 or acc is None:
        raise RuntimeError(f"reference run failed (rc {p.returncode}): {out[-500:]}")
    return {"align_s": wall - sum(setup), "wall_s": wall, "setup_s": sum(setup), "accepted": int(acc.group(1))}


if __name__ == "__main__":
    main()
