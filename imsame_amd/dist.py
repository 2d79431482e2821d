"""Multi-GPU sharding of the read set.

Reads are independent given the global chunk heads (fixed by -n_threads and
the full query, IMSAME.c:414), so one query is split into contiguous read
ranges, one per rank; every rank holds a replica of the index.  The only
collective is a reduction of a few counters (RCCL over xGMI with the "nccl"
backend, gloo on CPU in the tests).
"""
import numpy as np


def hip_runtimes():
    """Distinct HIP runtime files mapped into this process (/proc/self/maps).
    A multi-rank process must hold exactly one: torch's wheel ships
    libamdhip64 (SONAME libamdhip64.so.7, ROCm 7.0) and is imported first, so
    libimsame_dev.so's libamdhip64.so.7 dependency resolves to that same
    object by SONAME.  Loading the library first would map /opt/rocm's 7.2
    copy, and torch -- which asks for the FILE name libamdhip64.so -- would
    then map its own next to it: two runtimes in one process."""
    import os
    seen = set()
    try:
        for line in open("/proc/self/maps"):
            f = line.split()
            if len(f) >= 6 and os.path.basename(f[5]).startswith("libamdhip64"):
                seen.add(os.path.realpath(f[5]))
    except OSError:
        pass
    return sorted(seen)


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _kfd_gpu_nodes(nodes=KFD_NODES, dev_dri="/dev/dri"):
    """GPU agents of the KFD topology in the order the ROCm runtime numbers
    them (ascending node id; CPU nodes have simd_count 0), as (node, unique_id)
    pairs -- only those whose render node this process may open (a container
    lists every GPU of the host in sysfs but gets only its own /dev/dri
    devices; opening a render node starts no HIP runtime)."""
    import os
    out = []
    try:
        ids = sorted(int(d) for d in os.listdir(nodes) if d.isdigit())
    except OSError:
        return out
    for nid in ids:
        props = {}
        try:
            for line in open(os.path.join(nodes, str(nid), "properties")):
                f = line.split()
                if len(f) == 2:
                    props[f[0]] = f[1]
        except OSError:
            continue
        if int(props.get("simd_count", "0") or 0) <= 0:
            continue
        minor = props.get("drm_render_minor")
        if minor is not None and dev_dri is not None:
            try:
                os.close(os.open(os.path.join(dev_dri, "renderD%s" % minor), os.O_RDWR | os.O_CLOEXEC))
            except OSError:
                continue
        out.append((nid, props.get("unique_id", "")))
    return out


def _apply_visible(ids, spec, uuid_of=None):
    """A *_VISIBLE_DEVICES list applied to the devices `ids` (in order): the
    listed ordinals (or, with uuid_of, GPU-<hex unique id> entries) in list
    order, up to the first entry that names no device (the runtimes stop
    there); an empty value hides every device."""
    if spec is None:
        return list(ids)
    out = []
    for tok in spec.split(","):
        tok = tok.strip()
        k = None
        if tok.isdigit() and int(tok) < len(ids):
            k = int(tok)
        elif uuid_of is not None and tok.upper().startswith("GPU-"):
            try:
                want = int(tok[4:], 16)
            except ValueError:
                want = None
            k = next((i for i, d in enumerate(ids) if want is not None and uuid_of(d) == want), None)
        if k is None or ids[k] in out:
            break
        out.append(ids[k])
    return out


def visible_gpus(environ=None, nodes=KFD_NODES, dev_dri="/dev/dri"):
    """GPUs this process may use, counted WITHOUT torch or HIP: the rank
    launcher (bench.py --gpus N) forks its children afterwards, and a parent
    that had started the HIP runtime must not fork+exec them.  The KFD
    topology gives the GPU agents; ROCR_VISIBLE_DEVICES (ordinals or GPU-<uuid>,
    applied by the ROCm runtime first), then HIP_VISIBLE_DEVICES or
    CUDA_VISIBLE_DEVICES (ordinals among those) filter them."""
    import os
    env = os.environ if environ is None else environ
    gpus = _kfd_gpu_nodes(nodes, dev_dri)
    uid = {n: int(u) for n, u in gpus if u.isdigit()}        # KFD: decimal; ROCR: GPU-<hex>
    ids = _apply_visible([n for n, _ in gpus], env.get("ROCR_VISIBLE_DEVICES"), uuid_of=uid.get)
    hip = env.get("HIP_VISIBLE_DEVICES", env.get("CUDA_VISIBLE_DEVICES"))
    return len(_apply_visible(ids, hip))


def host_threads_per_rank(usable, world):
    """Host threads one rank of `world` may keep busy out of the `usable` CPUs
    of the job: an equal share, at least 2 (a lane thread and the caller)."""
    return max(2, int(usable) // max(1, int(world)))


def shard_range(n_reads, rank, world):
    """Contiguous [from, to) of rank `rank` out of `world`."""
    return (n_reads * rank) // world, (n_reads * (rank + 1)) // world


def _device_for_backend():
    import torch
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_reduce(values, op="sum"):
    """Reduce a short list of numbers across ranks (one collective)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=_device_for_backend())
    dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)
    return [float(x) for x in t.cpu().tolist()]


def align_sharded(align_fn, n_reads, rank, world, n_threads):
    """Run align_fn(read_from, read_to, n_threads) -> per-read results on this
    rank's shard; returns (results, (from, to), [accepted_total, reads_total])."""
    a, b = shard_range(n_reads, rank, world)
    res = align_fn(a, b, n_threads)
    acc = int(np.count_nonzero(res["status"] == 1))
    tot = all_reduce([acc, b - a])
    return res, (a, b), [int(tot[0]), int(tot[1])]


# ---------------------------------------------------------------------------
# Database shards (SURVEY 8(f) row 4 across GPUs): each rank holds one slice
# of the DATABASE (whole records; rank 0 the highest records, so a bucket's
# hits run rank 0, 1, ... in the reference's LIFO order, IMSAME.c:255-276)
# and aligns every read against it with imsame_dev_align_windows.  The
# reference's first accepted pair of a read is the accepted result with the
# smallest (window, rank) key: one min all-reduce of the keys, then one sum
# all-reduce of the winning 64-byte result rows.  The exchange is real data
# (16 B + 64 B per read) -- this is the path's one collective step.
# ---------------------------------------------------------------------------
NO_KEY = np.iinfo(np.int64).max


def db_shard_records(db_starts, db_len, rank, world):
    """Record range [lo, hi) of database shard `rank`: contiguous, top down
    (rank 0 = the highest records), cut at record starts near equal bases."""
    st = np.asarray(db_starts, dtype=np.uint64)
    n = len(st)
    # cut c (0 < c < world) at the first record starting at or after c/world of the bases
    cuts = [int(np.searchsorted(st, (db_len * c) // world)) for c in range(1, world)]
    edges = [0] + cuts + [n]                        # bottom-up record edges
    k = world - 1 - rank                            # rank 0 takes the top range
    return edges[k], edges[k + 1]


def shard_keys(res, win, rank, world):
    """Per-read key of this shard's result: window * world + rank if accepted.
    An accepted row always carries the window of its hit
    (imsame_dev_align_windows); ~0 there would make a negative key win the
    min, so it is refused (the C sliced path refuses it with IMSAME_E_STATE)."""
    acc = res["status"] == 1
    w = np.asarray(win, dtype=np.uint64)
    if np.any(w[acc] >= np.uint64(1) << np.uint64(62)):
        raise ValueError("accepted read without the window of its hit")
    return np.where(acc, (w.astype(np.int64) * world + rank), NO_KEY).astype(np.int64)


def merge_shard_results(parts):
    """Host merge of shard results [(res, win, rec_lo)] listed rank 0 first:
    per read, the accepted row with the smallest (window, rank); reads no
    shard accepted keep rank 0's row.  db_seq becomes global."""
    world = len(parts)
    keys = np.stack([shard_keys(r, w, k, world) for k, (r, w, _) in enumerate(parts)])
    best = keys.argmin(axis=0)
    out = parts[0][0].copy()
    for k, (r, _, lo) in enumerate(parts):
        m = (best == k) & (keys[k] != NO_KEY)
        out[m] = r[m]
        out["db_seq"][m] += lo
    return out


def merge_db_sharded(res, win, rec_lo, rank, world):
    """merge_shard_results over torch.distributed ranks (RCCL "nccl" on
    GPUs, gloo on CPU): min all-reduce of the keys, sum all-reduce of the
    winning rows (64 B each, so exactly one rank contributes a row).
    The merged rows are the per-read results; their path_off/path_len point
    into the WINNING rank's path arena, so .align text is rendered by that
    rank (or after gathering its paths), not from the merged rows alone."""
    import torch
    import torch.distributed as dist
    dev = _device_for_backend()
    key = shard_keys(res, win, rank, world)
    kmin = torch.from_numpy(key.copy()).to(dev)
    dist.all_reduce(kmin, op=dist.ReduceOp.MIN)
    kmin = kmin.cpu().numpy()
    mine = (kmin == key) & (key != NO_KEY)
    rows = res.copy()
    rows["db_seq"] += np.where(mine, rec_lo, 0).astype(rows["db_seq"].dtype)
    contrib = mine | ((kmin == NO_KEY) & (rank == 0))
    rows[~contrib] = np.zeros(1, dtype=rows.dtype)
    words = torch.from_numpy(rows.view(np.int64).copy()).to(dev)
    dist.all_reduce(words, op=dist.ReduceOp.SUM)
    return words.cpu().numpy().view(res.dtype).reshape(res.shape)
