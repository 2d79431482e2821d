#!/usr/bin/env python3
"""Benchmark of the IMSAME seed-and-extend hot path on MI355X.

Metric (BASELINE.json): reads aligned/sec (node), 1M x 150 bp synthetic
Illumina-like reads vs a 50 Mbp synthetic reference (configs[1]), at 1, 2, 4
and 8 GPUs.

One step = the rank's shard of the query uploaded (H2D from page-locked host
memory) + one imsame_dev_align pass over it (seed scan + ungapped/e-value +
NW wavefront + backtrack + acceptance + D2H of the per-read results).
N GPUs (strong scaling, the default): one process per GPU (torchrun); the
1M-read query is cut into N contiguous shards (imsame_amd.dist.shard_range),
each rank aligns its shard against its replica of the index with the chunk
heads of -n_threads over the WHOLE query, so the union of the shards is
exactly the single-GPU run; the only collective is an RCCL all-reduce of the
clock (max) and the accepted count.  value = 1M * steps / max-over-ranks wall
time of the timed region.  --scaling weak gives every rank its own 1M reads.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c5|c5w]
"""
import argparse
import ctypes as C
import json
import os
import platform
import sys
import time

import numpy as np

# one hardware queue per alignment lane: HIP maps a process's streams onto
# GPU_MAX_HW_QUEUES queues (4 on the GPU boxes when unset), two lanes on one
# queue serialize, and the library runs at most one lane per queue
# (imsame_dev.hip:lanes_for_queues; it never sets the variable itself).  The
# benchmark, as a host program, asks for 8 before anything starts HIP (torch
# does in a multi-rank run); results do not depend on it.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
from imsame_amd.dist import host_threads_per_rank  # noqa: E402  (numpy only: no torch, no HIP)

METRIC = "reads aligned/sec (node), 1M×150bp vs 50Mbp ref, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md, chip-level parameters


# BASELINE.json configs (SURVEY 8(d) canonical inputs).  c2 is the metric's
# configuration and the default; c3 is configs[2]'s per-GPU shard (10M reads /
# 8 GPUs vs 500 Mbp); c5 is configs[4] (ONT-like 10 kbp reads, raised
# MAX_READ_SIZE, reads capped by --reads); c5w the same reads vs long records.
CONFIGS = {
    "c2": dict(reads=1_000_000, read_len=150, ref_bp=50_000_000, record_bp=2_000, ont=False, max_rs=None,
               cpu_sample=40_000, seeds=(42, 43),
               workload="C2: 1M x 150 bp Illumina-like reads vs 50 Mbp synthetic reference "
                        "(2 kbp records), BASELINE.json configs[1]"),
    "c3": dict(reads=1_250_000, read_len=150, ref_bp=500_000_000, record_bp=2_000, ont=False, max_rs=None,
               cpu_sample=4_000, seeds=(43, 44),
               workload="C3 per-GPU shard: 1.25M x 150 bp reads per GPU (10M over 8) vs 500 Mbp synthetic "
                        "reference (2 kbp records), BASELINE.json configs[2]"),
    "c5": dict(reads=100_000, read_len=10_000, ref_bp=50_000_000, record_bp=2_000, ont=True, max_rs=10_001,
               cpu_sample=0, seeds=(42, 48),
               workload="C5: 10 kbp ONT-like reads (5% sub, 2.5% ins, 2.5% del) vs 50 Mbp synthetic reference, "
                        "MAX_READ_SIZE raised to 10001, BASELINE.json configs[4] (2 kbp records: every hit is "
                        "rejected a priori, seed scan only)"),
    # C5 against records long enough to hold a read: the long-read NW runs
    # (10 kbp x 12 kbp = 120M cells per candidate, the packed long-read kernel)
    "c5w": dict(reads=4_096, read_len=10_000, ref_bp=50_004_000, record_bp=12_001, ont=True, max_rs=12_001,
                cpu_sample=0, seeds=(42, 48),
                workload="C5w: 10 kbp ONT-like reads vs 50 Mbp synthetic reference in 12,001 bp records, "
                         "MAX_READ_SIZE raised to 12001 (BASELINE.json configs[4] shape with records that "
                         "can hold a read, so the long-read NW runs)"),
}


def nw_kernel_name(read_len, record_bp, igap=-5, egap=-2):
    """The NW kernel imsame_dev.hip:plan_nw picks for this shape (mirror of
    nw16_kernel.hip:nw16_fits for the default gap parameters)."""
    if read_len > 160:
        if igap > 0 or egap > 0:
            return "nw_kernel"
        # nwp_kernel.hip:nwp_fits (2 NWP_S2 + |ig| + |eg| (L + 64) + 116 <= 32767): packed
        # pairs, else the int32 nwl_kernel.hip
        fits = -igap <= 1024 and -egap <= 16 and 2 * 2308 - igap - egap * (max(read_len, record_bp) + 64) + 116 <= 32767
        return "nwp_kernel" if fits else "nwl_kernel"
    if igap > 0 or egap > 0:
        return "nw_kernel"
    ycols = -(-read_len // 10) * 10
    R = 4 * ycols - igap - egap * (record_bp + 64 + ycols + 2) + 16
    return "nw16_kernel" if R <= 8191 else "nw_kernel"


def nw16_form(read_len, record_bp):
    """The packed kernel's column form at this shape (imsame_dev.hip:plan_nw,
    nw16_kernel.hip): the 19-column form when every read has 150 bases and 8
    groups fit the LDS, else 10 columns per lane."""
    if read_len == 150 and 8 * ((record_bp + 15) // 16 * 16) <= 16384:
        K, G, GPW = 19, 8, 8
    else:
        K = 10
        G = -(-read_len // K)
        GPW = max(1, min(64 // G, 16384 // ((max(record_bp, 2) + 15) // 16 * 16)))
    nrec = 2 if K <= 8 else 3 if K <= 10 else 2 * ((K + 7) // 8)
    return {"K": K, "G": G, "GPW": GPW, "nst": 4 * K + 5, "nrec": nrec, "ck": 32 if K <= 5 else 48}


def nw16_min_bytes_per_cell(read_len, record_bp):
    """HBM bytes per DP cell the TWO-PASS kernel cannot avoid:
    every wave writes its register checkpoint (4K+5 dwords per lane) every CK
    steps, the traceback of the band the walk reads (the first sweep's
    predicted window: the read's rows + 32 above + 24 below + the skew G, NREC
    dwords per lane per step), and reads the record and the read once.
    Per DP cell of the wave's 2 x GPW candidates."""
    f = nw16_form(read_len, record_bp)
    steps = record_bp + f["G"]
    cells_per_wave_step = 2 * f["GPW"] * read_len * record_bp / steps
    ck = f["nst"] * 4 * 64 / f["ck"]
    band = read_len + 32 + 24 + f["G"]
    tb = f["nrec"] * 4 * 64 * band / steps
    inp = (record_bp + read_len) / (record_bp * read_len)
    bpc = (ck + tb) / cells_per_wave_step + inp
    return {"bytes_per_cell": round(bpc, 4), "checkpoint": round(ck / cells_per_wave_step, 4),
            "band_traceback": round(tb / cells_per_wave_step, 4), "inputs": round(inp, 5), "form": f}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2",
                    help="BASELINE.json workload (c2 = the metric's config; c3/c5/c5w are stress runs)")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong: ONE query of --reads reads split over the ranks (the metric); "
                         "weak: every rank its own --reads reads")
    ap.add_argument("--reads", type=int, default=None, help="reads in the query (weak: per rank)")
    ap.add_argument("--read-len", type=int, default=None)
    ap.add_argument("--ref-bp", type=int, default=None)
    ap.add_argument("--record-bp", type=int, default=None)
    ap.add_argument("--n-threads", type=int, default=16, help="reference -n_threads semantics")
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="reads in the CPU baseline sample (0: skip; default: the config's)")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="threads of the CPU baseline (default: the host cores this process may use)")
    ap.add_argument("--cpu-kind", choices=("auto", "port", "reference"), default="auto",
                    help="auto: the compiled reference (oracle/_ref/IMSAME) when present, else the port")
    ap.add_argument("--slice-bases", type=int, default=0,
                    help="search the database in slices of at most this many bases, one slice's index in HBM "
                         "at a time (imsame_dev_align_sliced; the index rebuilds are inside the timed step)")
    ap.add_argument("--e2e", choices=("auto", "on", "off"), default="auto",
                    help="end-to-end imsame CLI run (parse, index, align, render, write) after the timed steps "
                         "(auto: on for c2 at N=1)")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo: rehearsal on one card)")
    ap.add_argument("--dist", action="store_true",
                    help="initialise torch.distributed (--dist-backend) even at one rank, so the collectives of an "
                         "N-rank run (RCCL all-reduce of the clock and counters) execute next to the library's streams")
    ap.add_argument("--device", type=int, default=None,
                    help="HIP device of this rank (default LOCAL_RANK; a fixed value rehearses N ranks on one card)")
    ap.add_argument("--device-count-override", type=int, default=None, metavar="N",
                    help="rehearsal: the --gpus launcher takes N GPUs as visible (counted without HIP it sees "
                         "fewer) and rank r uses device LOCAL_RANK mod the real count")
    ap.add_argument("--shard", default=None, metavar="R/N",
                    help="diagnostic: on one GPU, time only rank R's shard of an N-GPU strong-scaling run")
    ap.add_argument("--upload", choices=("async", "sync"), default="async",
                    help="query H2D per step: queued in parts that each lane waits for (async) or waited for "
                         "before the alignment (sync); inside the timed step either way")
    ap.add_argument("--traffic-json", default=None, help="PMC bytes per cell (default profiles/nw_traffic[_CONFIG].json)")
    ap.add_argument("--valu-json", default=None, help="PMC VALU per cell (default profiles/nw_valu[_CONFIG].json)")
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    for k in ("reads", "read_len", "ref_bp", "record_bp", "cpu_sample"):
        if getattr(a, k) is None:
            setattr(a, k, cfg[k])
    sfx = "" if a.config == "c2" else "_" + a.config       # scripts/pmc_r2.py writes them per config
    a.traffic_json = a.traffic_json or os.path.join(REPO, "profiles", f"nw_traffic{sfx}.json")
    a.valu_json = a.valu_json or os.path.join(REPO, "profiles", f"nw_valu{sfx}.json")
    return a


def host_cpu():
    """The host this process runs on: model, online CPUs (nproc), the CPUs it
    may run on (affinity) and its cgroup CPU quota; `usable` is what the CPU
    baseline gets (the GPU box gives a process a share of a larger host)."""
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        usable = min(usable, int(env))
    return {"model": model, "nproc": nproc, "affinity": aff, "cgroup_quota_cpus": quota, "usable": usable}


def launch_ranks(a):
    """`--gpus N` without a launcher: start N rank processes of this script,
    one per GPU -- the fan-out IMSAME does with pthread_create over read
    ranges (IMSAME.c:414-467), one process per GPU here -- with RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT set as torch.distributed.run
    sets them.  The parent never touches the GPU (children are fresh
    processes, not forks of a HIP process).  Rank 0 prints the line (the
    children share this stdout); a failing rank stops the others and its exit
    status becomes ours."""
    import signal
    import socket
    import subprocess
    from imsame_amd.dist import visible_gpus           # KFD topology + *_VISIBLE_DEVICES: no torch, no HIP
    n_real = visible_gpus()
    if a.device is None:
        n = a.device_count_override if a.device_count_override is not None else n_real
        if a.gpus > n:
            sys.exit(f"bench.py: --gpus {a.gpus} but {n} GPU(s) visible (--device D rehearses N ranks on one card)")
        if a.device_count_override is not None and n_real < 1:
            sys.exit("bench.py: --device-count-override needs at least one visible GPU")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   IMSAME_BENCH_LAUNCHED="1", IMSAME_BENCH_VISIBLE=str(n_real))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                r = p.poll()
                if r is None:
                    continue
                live.remove(p)
                if r != 0 and rc == 0:
                    rc = r if r > 0 else 128 - r
                    for q in live:                       # the collectives would wait for the dead rank
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    gpu = local if a.device is None else a.device
    if a.device is None and a.device_count_override is not None:       # rehearsal: ranks share the real cards
        gpu = local % max(1, int(os.environ.get("IMSAME_BENCH_VISIBLE", "1")))
    # host threads of this rank: an equal share of the job's usable CPUs
    # (upload host pass, imsame_dev.hip:host_threads_cap); set before the
    # library is loaded (it reads the variable once)
    hc = host_cpu()
    threads = host_threads_per_rank(hc["usable"], world)
    os.environ.setdefault("IMSAME_HOST_THREADS", str(threads))
    backend = None
    if world > 1 or a.dist:
        import torch
        import torch.distributed as dist
        backend = a.dist_backend
        if world == 1 and "RANK" not in os.environ:          # --dist at one rank, no launcher
            import socket
            s_ = socket.socket()
            s_.bind(("127.0.0.1", 0))
            os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(s_.getsockname()[1]))
            s_.close()
        if backend == "nccl":
            torch.cuda.set_device(gpu)
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    import imsame_amd
    from imsame_amd.dist import shard_range, hip_runtimes
    from tests import synth

    # synthetic inputs: the reference is replicated; strong scaling = ONE query
    # (the metric's 1M reads) whose contiguous shards go to the ranks, with the
    # chunk heads of -n_threads over the whole query
    cfg = CONFIGS[a.config]
    ref, rst = synth.make_reference_arr(a.ref_bp, a.record_bp, seed=cfg["seeds"][0])
    gen = synth.make_long_reads_arr if cfg["ont"] else synth.make_reads_arr
    strong = a.scaling == "strong"
    q, qs = gen(ref, a.reads, a.read_len, seed=cfg["seeds"][1] + (0 if strong else 1000 * rank))
    lo, hi = shard_range(a.reads, rank, world) if strong else (0, a.reads)
    if a.shard and world == 1:                        # one rank's work of an N-GPU run, on one GPU
        sr, sn = (int(x) for x in a.shard.split("/"))
        lo, hi = shard_range(a.reads, sr, sn)
    dev = imsame_amd.Device(gpu)
    t0 = time.time()
    dev.index(ref, rst)
    t_index = time.time() - t0
    pin = imsame_amd.PinnedArray(len(q))              # page-locked source of the per-step upload
    pin.array[:] = q
    qp = pin.array
    rpin = imsame_amd.PinnedArray(hi - lo, imsame_amd.RESULT_DTYPE)   # page-locked results, reused
    params = dev.params(max_read_size=cfg["max_rs"]) if cfg["max_rs"] else dev.params()

    n_slices = 1
    h2d = []

    def step():
        nonlocal n_slices
        t = time.perf_counter()
        # H2D of this rank's shard, inside the step: queued in parts, each lane
        # of the alignment starts when its reads are in HBM (--upload async)
        dev.set_query(qp, qs, lo, hi, wait=a.upload == "sync")
        h2d.append(time.perf_counter() - t)
        if a.slice_bases:
            res, paths, st, n_slices = dev.align_sliced(ref, rst, a.slice_bases, n_threads=a.n_threads,
                                                        params=params, read_from=lo, read_to=hi)
            return res, paths, st
        return dev.align(lo, hi, n_threads=a.n_threads, params=params, out=rpin.array)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(a.warmup):
        step()
    h2d.clear()
    barrier()
    stats = []
    cpu0 = time.process_time()                      # this rank's host CPU seconds (all its threads)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res, _, st = step()
        stats.append(st.as_dict())
    barrier()
    elapsed = time.perf_counter() - t0
    host_cpu_s = (time.process_time() - cpu0) / a.steps
    accepted = int((res["status"] == 1).sum())
    res = res.copy()
    if dist is not None:
        from imsame_amd.dist import all_reduce     # RCCL: max of the clocks, sum of the counters
        elapsed = all_reduce([elapsed], op="max")[0]
        accepted_all = int(all_reduce([accepted])[0])
    else:
        accepted_all = accepted
    total_reads = (a.reads if strong else world * a.reads) * a.steps
    if a.shard and world == 1:
        total_reads = (hi - lo) * a.steps             # the shard's own rate (diagnostic line)
    value = total_reads / elapsed

    # dominant kernel: the NW launches.  Algorithmic bytes per NW candidate
    # (SURVEY 8(d)): record + read + 2 B/cell traceback floor; HIP events on
    # the library's own stream bracket every NW launch.
    nw_ms = sum(s["ms_nw"] for s in stats)                 # summed per-launch HIP-event durations
    nw_busy = sum(s["ms_nw_busy"] for s in stats)          # union of the launch intervals (lanes overlap)
    nw_launches = sum(s["nw_launches"] for s in stats)
    cells = sum(s["nw_cells"] for s in stats)
    n_nw = sum(s["n_nw"] for s in stats)
    seq_bytes = n_nw * (a.record_bp + a.read_len)
    alg_bytes = 2 * cells + seq_bytes
    # achieved: algorithmic bytes / the time the device ran NW launches.  The
    # lanes' launches overlap: the per-launch average (avg_launch_ms; what
    # rocprofv3 --stats reports per kernel: kernel_avg_launch_ms) times the
    # launches exceeds that time by launch_overlap (scripts/nw_busy.py
    # recomputes the union from the kernel trace)
    achieved = alg_bytes / (nw_busy / 1e3) / 1e9 if nw_busy else 0.0
    kernel = nw_kernel_name(a.read_len, a.record_bp)
    per_launch = alg_bytes / max(nw_launches, 1)
    traffic = bpc = None
    if os.path.exists(a.traffic_json):
        try:
            tj = json.load(open(a.traffic_json))
            if tj.get("kernel") == kernel and tj.get("config", "c2") == a.config:   # PMC pass of THIS kernel
                # bytes per DP cell of the PMC pass x this run's cells per launch
                # (launch sizes depend on the lane count; the per-cell rate does not)
                bpc = tj.get("hbm_bytes_per_cell")
                traffic = int(bpc * cells / max(nw_launches, 1)) if bpc else None
        except Exception:
            traffic = bpc = None
    cells_per_s = cells / (nw_busy / 1e3) if nw_busy else 0.0
    # launches of the dominant kernel alone (imsame_stats.launch_pk: packed
    # nw16_kernel vs the int32 nw_kernel that takes the small last launches),
    # the average rocprofv3 --stats reports for that kernel name
    # (launch_nwp: the packed long-read nwp_kernel vs the int32 nwl_kernel)
    kbits = "launch_nwp" if kernel in ("nwp_kernel", "nwl_kernel") else "launch_pk"
    pk_ms = [m for s_ in stats for j, m in enumerate(s_["launch_ms"])
             if ((s_.get(kbits, 0) >> j) & 1) == (1 if kernel in ("nw16_kernel", "nwp_kernel") else 0)]
    # HBM: the contract's algorithmic figure (2 B/cell), the
    # two-pass kernel's own minimum (nw16_min_bytes_per_cell) and the bytes
    # the PMC counters saw per cell
    measured = bpc * cells_per_s / 1e9 if bpc and cells_per_s else None
    tp = nw16_min_bytes_per_cell(a.read_len, a.record_bp) if kernel == "nw16_kernel" else None
    hbm = {"basis": "CONTRACT figure: algorithmic bytes of SURVEY 8(d) (xlen + ylen + 2 B/cell traceback floor per "
                    "NW) / NW busy time -- the kernel stores 4 bits per cell of a band, not 2 B per cell",
           "contract_achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "contract_frac": round(achieved / HBM_PEAK_GBS, 4),
           "two_pass_min": tp,
           "measured_bytes_per_cell": bpc,
           "measured_over_two_pass_min": round(bpc / tp["bytes_per_cell"], 3) if bpc and tp else None,
           "measured_gbs": round(measured, 2) if measured else None,
           "measured_frac": round(measured / HBM_PEAK_GBS, 4) if measured else None,
           "measured_basis": "PMC bytes per DP cell (2 x FETCH_SIZE + WRITE_SIZE, %s) x this run's cells/s of NW "
                             "busy time" % os.path.relpath(a.traffic_json, REPO)}
    valu = valu_roofline(a.valu_json, kernel, a.config, cells_per_s, a.read_len, a.record_bp)
    common = {"traffic": traffic,
              "traffic_over_alg": round(traffic / per_launch, 4) if traffic and per_launch else None,
              "kernel": kernel, "launches": nw_launches,
              "nw_fallback": sum(s_.get("nw_fallback", 0) for s_ in stats),
              "avg_launch_ms": round(nw_ms / max(nw_launches, 1), 4),
              "kernel_launches": len(pk_ms),
              "kernel_avg_launch_ms": round(sum(pk_ms) / max(len(pk_ms), 1), 4),
              "nw_busy_ms_per_step": round(nw_busy / a.steps, 3),
              "launch_overlap": round(nw_ms / nw_busy, 3) if nw_busy else None,
              "alg_bytes_per_launch": int(per_launch),
              "cells_per_s": round(cells_per_s, 1)}
    if valu:
        # the NW kernel's binding resource is VALU issue: the
        # headline bound; the contract's HBM figure stays under "hbm"
        roofline = dict({"bound": "valu", "achieved": valu["achieved"], "peak": valu["issue_peak"],
                         "unit": valu["unit"], "frac": valu["frac"]}, **common, valu=valu, hbm=hbm)
    else:
        roofline = dict({"bound": "hbm", "achieved": hbm["contract_achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": hbm["contract_frac"]}, **common, valu=None, hbm=hbm)

    cpu = parity = None
    if rank == 0 and world == 1 and a.cpu_sample > 0:
        # the oracle as the checker: the timed run's own rows on three windows
        parity = timed_parity(ref, rst, q, qs, res, lo, hi, a, params)
        if a.slice_bases:
            dev.index(ref, rst)                     # the sample is checked against the whole index
        cpu = cpu_baseline(dev, ref, rst, q, qs, a, params)

    e2e = None
    if rank == 0 and world == 1 and (a.e2e == "on" or (a.e2e == "auto" and a.config == "c2")):
        dev.close()                                 # the CLI opens the device itself
        e2e = run_e2e(ref, rst, q, qs, a)

    if rank == 0:
        last = stats[-1]
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "reads/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": a.scaling, "vs_baseline": None,
            "dtype": "int16" if kernel in ("nw16_kernel", "nwp_kernel") else "int32", "data": "synthetic",
            "config": {"workload": cfg["workload"] + (f"; {a.reads} reads total over {world} GPU(s), contiguous "
                                                      f"shards" if strong else f"; {a.reads} reads per GPU")
                       + (f"; database searched in {n_slices} slices of <= {a.slice_bases} bases"
                          if a.slice_bases else ""),
                       "reads": a.reads, "reads_per_gpu": hi - lo, "read_len": a.read_len, "ref_bp": a.ref_bp,
                       "record_bp": a.record_bp, "n_threads_semantic": a.n_threads,
                       "parallelism": f"dp{world} (read shards, replicated index)"
                       + (f"; collectives: {'RCCL' if backend == 'nccl' else backend} over {world} rank(s)"
                          if backend else "")
                       + ("" if world == 1 or a.dist_backend == "nccl" else
                          f"; REHEARSAL: {a.dist_backend} collectives, device {gpu} shared by all ranks")},
            "roofline": roofline,
            "seed_roofline": seed_roofline(last, hi - lo, a.read_len),
            "parity": parity,
            "cpu_baseline": cpu,
            "e2e": e2e,
            "ranks": {"world": world, "backend": ("rccl" if backend == "nccl" else backend),
                      "device": gpu, "host_cpus_usable": hc["usable"],
                      "host_threads_per_rank": int(os.environ["IMSAME_HOST_THREADS"]),
                      "host_cpu_s_per_step": round(host_cpu_s, 5),
                      "host_cpu_s_per_step_basis": "rank 0's process CPU time (user + system, every thread: the "
                                                   "lanes' host threads, the upload pass, waits) over the timed "
                                                   "steps / steps",
                      "lane_wait": os.environ.get("IMSAME_WAIT", "yield"),
                      "launcher_visible_gpus": (int(os.environ["IMSAME_BENCH_VISIBLE"])
                                                if "IMSAME_BENCH_VISIBLE" in os.environ else None),
                      "launcher": "bench.py" if os.environ.get("IMSAME_BENCH_LAUNCHED") else
                                  ("torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ or world > 1
                                   else None),
                      "hip_runtime": hip_runtimes()},
            "detail": {"accepted_reads": accepted_all, "index_build_s": round(t_index, 3),
                       "rounds": last["rounds"], "nw_per_read": round(last["n_nw"] / max(hi - lo, 1), 4),
                       "hits_per_read": round(last["n_hits"] / max(hi - lo, 1), 2),
                       "ms_h2d_query": round(1e3 * sum(h2d) / max(len(h2d), 1), 3), "upload": a.upload,
                       "nw_cells": last["nw_cells"], "n_nw": last["n_nw"],
                       "lanes": last["lanes"], "nw_redo_waves": last.get("nw_redo"),
                       "nw_window_walks": last.get("nw_win"),
                       "ms_seed": round(last["ms_seed"], 3), "ms_nw": round(last["ms_nw"], 3),
                       "ms_nw_busy": round(last["ms_nw_busy"], 3),
                       "ms_nw_first_start": round(last["ms_nw_first"], 3),
                       "ms_nw_last_end": round(last["ms_nw_last"], 3),
                       "ms_align_call": round(last["ms_total"], 3),
                       "ms_host_setup": round(last["ms_setup"], 3), "ms_d2h_results": round(last["ms_d2h"], 3),
                       "nw_accounting": nw_accounting(last, hi - lo, parity),
                       "nw_launch_cand": last["launch_cand"],
                       "nw_launch_ms": [round(x, 3) for x in last["launch_ms"]]},
        }
        print(json.dumps(line), flush=True)
    dev.close()
    pin.free()
    rpin.free()
    if dist is not None:
        dist.destroy_process_group()


def nw_accounting(st, n_reads, parity):
    """The device's NW work against the reference's (alignmentFunctions.c:
    126-186 runs one NW per e-value-passing hit, in visiting order, until one
    is accepted).  Device: n_nw = the distinct (read, record) pairs up to each
    read's accepted one -- the reference's work without its repeats of an
    already rejected record -- plus `spec_extra`, the candidates a read
    emitted past its accepted one (speculation, round_policy.h), counted by
    update_kernel.  Oracle on the parity windows (when the checker ran): the
    same distinct count, and the reference's own count with the repeats."""
    n = max(n_reads, 1)
    waste = st.get("nw_spec_waste", 0)
    out = {"nw_per_read": round(st["n_nw"] / n, 4), "spec_extra_per_read": round(waste / n, 4),
           "needed_per_read": round((st["n_nw"] - waste) / n, 4),
           "spec_extra_frac": round(waste / max(st["n_nw"], 1), 4)}
    if parity and parity.get("oracle_nw_distinct") is not None:
        m = max(parity["reads_compared"], 1)
        out["windows_oracle_distinct_per_read"] = round(parity["oracle_nw_distinct"] / m, 4)
        if parity.get("oracle_nw_reference") is not None:
            out["nw_ref_per_read"] = round(parity["oracle_nw_reference"] / m, 4)
    return out


def seed_roofline(st, n_reads, read_len):
    """The seed scan's memory work against its kernels' own time (SURVEY
    8(d)): per read its bases, per probed window two CSR offsets, per CSR
    entry read the entry, per ungapped extension the database and query bytes
    it loads (16-byte chunk pairs), counted by the kernels
    (imsame_stats.seed_*).  Time = the seed launches' HIP-event durations
    summed over lanes (they share the chip with NW launches of other lanes).
    The scan is a chain of dependent random probes (offsets -> entries ->
    record bytes), so the rate it reaches is latency-bound: `probes_per_s`
    and `bytes_per_probe` are the model, the HBM fraction is context."""
    wins, ents, ch = st.get("seed_windows", 0), st.get("seed_entries", 0), st.get("seed_ext_chunks", 0)
    ms = st.get("ms_seed", 0.0)
    if not wins or not ms:
        return None
    survey = n_reads * read_len + 8 * wins + 4 * st["n_hits"] + 32 * ch       # SURVEY 8(d) widths
    # as built: u64 bucket offsets, 8-byte entries, and per 16-base chunk pair
    # of an extension one packed dword of the database and one of the query
    # (seed_kernel.hip:ungapped_raw on 2-bit codes)
    built = n_reads * read_len + 16 * wins + 8 * ents + 8 * ch
    t = ms / 1e3
    return {"bound": "latency (dependent random probes)", "kernel_ms": round(ms, 3),
            "windows": wins, "entries": ents, "hits": st["n_hits"], "ext_chunk_pairs": ch,
            "bytes_survey_model": survey, "bytes_as_built": built,
            "achieved_gbs": round(built / t / 1e9, 2), "peak_gbs": HBM_PEAK_GBS,
            "frac": round(built / t / 1e9 / HBM_PEAK_GBS, 4),
            "probes_per_s": round(wins / t, 1), "entries_per_s": round(ents / t, 1),
            "bytes_per_probe": round(built / wins, 2),
            "ext_bytes_per_hit": round(8 * ch / max(st["n_hits"], 1), 1),
            "ext_form": "2-bit packed database and query, 16 bases per dword"}


# MI355X_MICROARCH.md: a wave issues one VALU instruction over 2 cycles
# (64 lanes on a SIMD-32), 4 SIMDs x 256 CUs at 2.4 GHz
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2.0     # wave-instructions / s


def valu_roofline(path, kernel, config, cells_per_s, read_len=150, record_bp=2000):
    """The NW kernel's binding resource is VALU issue.  Lane-
    instructions per cell come from a PMC pass (SQ_INSTS_VALU x 64 / cells of
    the same launches, profiles/nw_valu.json); achieved issue = that x the
    cells/s measured here / 64, against the 2-cycle issue peak."""
    if not os.path.exists(path):
        return None
    try:
        vj = json.load(open(path))
    except Exception:
        return None
    if vj.get("kernel") != kernel or vj.get("config", "c2") != config:
        return None
    ipc = vj["lane_instr_per_cell"]
    rate = ipc * cells_per_s / 64.0
    out = {"instr_per_cell": round(ipc, 3), "achieved": round(rate / 1e9, 2), "issue_peak": round(VALU_ISSUE_PEAK / 1e9, 2),
           "unit": "G wave-instr/s", "frac": round(rate / VALU_ISSUE_PEAK, 4), "source": os.path.relpath(path, REPO),
           "note": "peak = 2 cycles per wave instruction at 2.4 GHz; v_pk_*_i16 / v_perm issue at ~4 "
                   "(profiles/r06_valu_rate.txt)"}
    # the shader clock under this config's NW load (profiles/nw_clock.json:
    # s_memtime / s_memrealtime in the bench's own launches) and the issue
    # fraction at that clock instead of the 2.4 GHz peak
    kp = os.path.join(REPO, "profiles", "nw_clock.json")
    if os.path.exists(kp):
        try:
            kj = json.load(open(kp))
            if kj.get("kernel") == kernel and config in kj:
                ghz = kj[config]["shader_clock_ghz"]
                out.update({"shader_clock_ghz": ghz,
                            "frac_at_measured_clock": round(rate / (VALU_ISSUE_PEAK * ghz / 2.4), 4),
                            "clock_source": os.path.relpath(kp, REPO)})
        except Exception:
            pass
    # the measured ceiling of this instruction mix: the first-sweep loop
    # alone on a full chip (scripts/micro/nw16_loop.py), cycles per VALU per
    # SIMD -> a fraction of the same 2-cycle peak
    cp = os.path.join(REPO, "profiles", "nw16_loop_ceiling.json")
    if os.path.exists(cp):
        try:
            cj = json.load(open(cp))
            if cj.get("kernel") == kernel and cj.get("form") == nw16_form(read_len, record_bp)["K"]:
                out.update({"mix_ceiling_frac": cj["mix_ceiling_frac"],
                            "mix_ceiling_cycles_per_valu": cj["cycles_per_valu_per_simd"],
                            "frac_of_mix_ceiling": round(out["frac"] / cj["mix_ceiling_frac"], 4),
                            "mix_ceiling_source": os.path.relpath(cp, REPO)})
        except Exception:
            pass
    return out


def run_e2e(ref, rst, q, qs, a):
    """The whole imsame command on the same inputs written as FASTA: parse,
    index, upload, align, render + write of the .align (SURVEY 8(d)
    end-to-end wall; the reference's phases IMSAME.c:102,295,407,470).  The
    CLI prints a JSON phase line on stderr."""
    import re
    import shutil
    import subprocess
    import tempfile
    from tests import synth
    cli = os.path.join(REPO, "imsame_amd", "bin", "imsame")
    if not os.access(cli, os.X_OK):
        return None
    td = tempfile.mkdtemp(prefix="imsame_e2e_")
    try:
        dbf, qf, outf = os.path.join(td, "db.fa"), os.path.join(td, "q.fa"), os.path.join(td, "out.align")
        synth.write_fasta(dbf, ref, rst, "ref", width=80)
        synth.write_fasta(qf, q, qs, "read", width=0)
        free = shutil.disk_usage(td).free
        need = 4 * 1024 ** 3                         # ~3.3 KB of text per accepted read at C2
        out = outf if free > need else "/dev/null"
        extra = os.environ.get("IMSAME_E2E_ARGS", "").split()          # experiments, e.g. -batch_reads N
        env = dict(os.environ, IMSAME_T_LAUNCH="%.6f" % time.time())   # the CLI reports main entry / exit from it
        t0 = time.monotonic()
        p = subprocess.run([cli, "-query", qf, "-db", dbf, "-out", out, "-n_threads", str(a.n_threads)] + extra,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=900, env=env)
        wall = time.monotonic() - t0
        if os.environ.get("IMSAME_E2E_LOG"):                            # diagnostics: the CLI's stderr
            with open(os.path.join(REPO, "gpurun_out", os.environ["IMSAME_E2E_LOG"]), "wb") as f:
                f.write(p.stderr)
        m = re.search(rb"\[imsame\] phases (\{.*\})", p.stderr)
        if p.returncode != 0 or not m:
            return {"error": f"rc {p.returncode}: {p.stderr[-300:].decode(errors='replace')}"}
        ph = json.loads(m.group(1))
        tm = re.search(rb"\[imsame\] teardown (\{.*\})", p.stderr)          # device close after the phases line
        if tm:
            ph.update(json.loads(tm.group(1)))
        ph = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in ph.items()}
        if ph.get("exit_at_s", -1) >= 0:                # process start before main / exit after the last line
            ph["after_exit_s"] = round(wall - ph["exit_at_s"], 4)
        ph.update({"process_wall_s": round(wall, 3), "output": "file" if out == outf else "/dev/null (disk full)",
                   "output_fs": mount_fs(td), "cli_args": extra,
                   "reads_per_s_e2e": round(len(qs) / wall, 1),
                   "note": "imsame -query q.fa -db db.fa -out out.align -n_threads %d on one GPU; render+write of "
                           "finished batches overlaps the device's later batches; render_tail_s = exposed output "
                           "time after the last batch" % a.n_threads})
        return ph
    finally:
        shutil.rmtree(td, ignore_errors=True)


def timed_parity(ref, rst, q, qs, res, lo, hi, a, params):
    """Part of the CPU-baseline leg (the oracle as the checker, outside the
    timed region): the LAST TIMED STEP's own rows -- produced in exactly the
    mode that gives `value` (lanes, queues, async upload) -- against the oracle
    on three windows of the query (start, a -n_threads chunk head, end)."""
    from tests import parity as P
    from tests.oracle_bind import Oracle
    o = Oracle.load()
    po = o.params(max_read_size=params.max_read_size)
    t0 = time.time()
    out = P.check_windows(o, ref, rst, q, qs, res, lo, P.windows(lo, hi, len(qs), a.n_threads), a.n_threads, po,
                          count_ref=True)
    out["oracle_s"] = round(time.time() - t0, 2)
    out["rows_of"] = "the last timed step"
    return out


def mount_fs(path):
    """Filesystem type of the mount holding path (/proc/mounts, longest prefix)."""
    best, fs = "", None
    try:
        for line in open("/proc/mounts"):
            f = line.split()
            if len(f) > 2 and (path == f[1] or path.startswith(f[1].rstrip("/") + "/")) and len(f[1]) > len(best):
                best, fs = f[1], f[2]
    except OSError:
        pass
    return fs


def cpu_baseline(dev, ref, rst, q, qs, a, params):
    """The oracle (clean-room CPU restatement, 'port') on the host cores, on a
    bounded sample: the first cpu_sample reads of the rank-0 shard taken as a
    query of their own, -n_threads cpu_threads, alignment phase only (index
    build excluded, as for the GPU).  The GPU then aligns the same sample view
    with the same -n_threads and every per-read result is compared."""
    from tests.oracle_bind import Oracle
    from imsame_amd import PARITY_FIELDS
    hc = host_cpu()
    if a.cpu_threads is None:
        a.cpu_threads = hc["usable"]
    o = Oracle.load()
    n = min(a.cpu_sample, len(qs))
    qv = q[:int(qs[n])] if n < len(qs) else q
    po = o.params(max_read_size=params.max_read_size)
    rc, exp, _ = o.align(ref, rst, qv, qs[:n], po, a.cpu_threads)
    o.lib.or_last_align_seconds.restype = C.c_double
    secs = o.lib.or_last_align_seconds()
    dev.set_query(qv, qs[:n])
    got, _, _ = dev.align(0, n, n_threads=a.cpu_threads, params=params)
    host = dict(hc, threads_used=a.cpu_threads)
    same = int(np.all([exp[f] == got[f] for f in PARITY_FIELDS], axis=0).sum())
    port = {"value": round(n / secs, 1), "unit": "reads/s", "cores": a.cpu_threads, "kind": "port",
            "sample": f"first {n} reads of the rank-0 shard as their own query, oracle/imsame_oracle.c "
                      f"-n_threads {a.cpu_threads}, alignment-phase wall {secs:.2f} s",
            "sample_reads_identical_to_gpu": same, "sample_reads_compared": n, "host": host}
    ref_bin = os.path.join(REPO, "oracle", "_ref", "IMSAME")
    if a.cpu_kind == "port" or (a.cpu_kind == "auto" and not os.access(ref_bin, os.X_OK)):
        return port
    r = run_reference(ref_bin, ref, rst, qv, qs[:n], a.cpu_threads)
    gpu_acc = int((got["status"] == 1).sum())
    # the reference's own records vs the GPU rows (a second run with -out,
    # outside the timed one above)
    rows = reference_rows(ref_bin, ref, rst, qv, qs[:n], a.cpu_threads, got)
    return {"value": round(n / r["align_s"], 1), "unit": "reads/s", "cores": a.cpu_threads, "kind": "reference",
            "sample": f"first {n} reads of the rank-0 shard as their own query vs the same database, "
                      f"IMSAME compiled from the reference sources (oracle/Makefile ref, gcc -O3) -n_threads "
                      f"{a.cpu_threads}; alignment phase = process wall {r['wall_s']:.2f} s minus its single-threaded "
                      f"setup phases {r['setup_s']:.2f} s = {r['align_s']:.2f} s",
            "reference_accepted": r["accepted"], "gpu_accepted": gpu_acc,
            "reference_rows_identical": rows["identical"], "reference_rows_compared": rows["compared"],
            "reference_rows": rows, "host": host,
            "port": port}


def reference_rows(ref_bin, ref, rst, q, qs, threads, got):
    """Row-level parity with the compiled reference itself on the CPU-baseline
    sample: its `-out` file holds one record per accepted read, headed
    "(read, record) : id% cov% ylen" (alignmentFunctions.c:167; each header is
    one fprintf, so it survives the -n_threads interleave).  A read is
    identical when the reference accepted it and the GPU row has status 1,
    the same record, min(100, 100*identities/length) and min(100,
    100*length/ylen) in the reference's integer arithmetic, and the same ylen
    -- or when neither accepted it."""
    import re
    n = len(qs)
    ref_rows = {}
    dup = 0
    for m in re.finditer(rb"^\((\d+), (\d+)\) : (\d+)% (\d+)% (\d+)\n \$\$\$\$\$\$\$ $",
                         run_reference(ref_bin, ref, rst, q, qs, threads, want_out=True)["out"], re.M):
        k = int(m.group(1))
        dup += k in ref_rows
        ref_rows[k] = tuple(int(x) for x in m.groups()[1:])
    acc = got["status"] == 1
    ln = got["length"].astype(np.uint64)
    idp = np.minimum(100, (100 * got["identities"].astype(np.uint64)) // np.maximum(ln, 1))
    cov = np.minimum(100, (100 * ln) // np.maximum(got["ylen"].astype(np.uint64), 1))
    same = ~acc.copy()                                  # neither accepted ...
    for k, (sid, i_, c_, y_) in ref_rows.items():
        same[k] = bool(acc[k]) and (int(got["db_seq"][k]), int(idp[k]), int(cov[k]), int(got["ylen"][k])) == \
            (sid, i_, c_, y_)
    bad = np.flatnonzero(~same)
    return {"identical": int(same.sum()), "compared": n, "reference_records": len(ref_rows),
            "duplicate_headers": dup, "first_mismatches": [int(x) for x in bad[:5]],
            "fields": "read, record, id%, cov%, ylen of every '(read, record) : id% cov% ylen' header "
                      "(alignmentFunctions.c:167) vs the GPU row; reads without a header must have status != 1"}


def run_reference(ref_bin, ref, rst, q, qs, threads, want_out=False):
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
        outf = os.path.join(td, "out.align")
        t0 = time.monotonic()
        p = subprocess.run([ref_bin, "-db", dbf, "-query", qf, "-n_threads", str(threads)]
                           + (["-out", outf] if want_out else []),
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=600)
        wall = time.monotonic() - t0
        body = open(outf, "rb").read() if want_out and p.returncode == 0 else None
    out = p.stdout.decode(errors="replace")
    setup = [float(x) for x in re.findall(r"(?:Initialization took|building took|Took) ([0-9.eE+-]+) seconds", out)]
    acc = re.search(r"\[INFO\] (\d+) reads \(", out)
    if p.returncode != 0 or len(setup) != 3 or acc is None:
        raise RuntimeError(f"reference run failed (rc {p.returncode}): {out[-500:]}")
    return {"align_s": wall - sum(setup), "wall_s": wall, "setup_s": sum(setup), "accepted": int(acc.group(1)),
            "out": body}


if __name__ == "__main__":
    main()
