"""World-size-2 sharding on CPU (gloo): each rank aligns its read shard with
the kernel source (wave emulator) under the global chunk-head semantics; the
shards concatenate to the single-process oracle run and the counter
all-reduce matches it."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from imsame_amd import fasta, PARITY_FIELDS
from tests import golden_io as G


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case_name, T, out_dir):
    import torch.distributed as dist
    from imsame_amd.dist import align_sharded
    from tests.emu_bind import Emu
    from tests.oracle_bind import Oracle
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    case = G.e2e_case(case_name)
    db, dbs, brk = fasta.load(case["db"], True)
    q, qs, _ = fasta.load(case["query"])
    emu = Emu.load()
    p = Oracle.load().params()

    def fn(a, b, t):
        rc, res, _, _ = emu.align(db, dbs, q, qs, p, t, read_from=a, read_to=b, db_brk=brk)
        assert rc == 0
        return res

    res, (a, b), tot = align_sharded(fn, len(qs), rank, world, T)
    np.save(os.path.join(out_dir, f"r{rank}.npy"), res)
    np.save(os.path.join(out_dir, f"t{rank}.npy"), np.array(tot))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("T", [1, 3])
def test_two_rank_shards_equal_single_run(tmp_path, oracle, T):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), "reads_vs_reads", T, str(tmp_path)), nprocs=world, join=True)
    got = np.concatenate([np.load(tmp_path / f"r{r}.npy") for r in range(world)])
    case = G.e2e_case("reads_vs_reads")
    db, dbs, brk = fasta.load(case["db"], True)
    q, qs, _ = fasta.load(case["query"])
    rc, exp, _ = oracle.align(db, dbs, q, qs, None, T, brk)
    for f in PARITY_FIELDS:
        assert np.array_equal(got[f], exp[f]), f
    acc = int((exp["status"] == 1).sum())
    for r in range(world):
        assert list(np.load(tmp_path / f"t{r}.npy")) == [acc, len(qs)]


def _fake_parts(world, n=300, seed=3):
    """Per-shard results as imsame_dev_align_windows returns them (random
    accepts, windows in a small range so (window) ties across shards occur)."""
    from imsame_amd.abi import RESULT_DTYPE
    rng = np.random.default_rng(seed)
    ylen = rng.integers(50, 200, n)
    parts = []
    for k in range(world):
        r = np.zeros(n, dtype=RESULT_DTYPE)
        r["ylen"] = ylen
        acc = rng.random(n) < 0.4
        r["status"][acc] = 1
        for f in ("db_seq", "score", "bx", "by", "length", "identities", "head_x"):
            r[f][acc] = rng.integers(1, 1000, int(acc.sum()))
        win = np.where(acc, rng.integers(11, 20, n), np.iinfo(np.uint64).max).astype(np.uint64)
        parts.append((r, win, 1000 * (world - 1 - k)))          # rank 0 holds the top records
    return parts


def test_db_shard_merge_rule():
    """Smallest (window, shard) wins; a window tie goes to the higher records
    (lower rank: earlier in the LIFO bucket); unaccepted reads keep shard 0's
    row; db_seq becomes global."""
    from imsame_amd.dist import merge_shard_results, db_shard_records
    parts = _fake_parts(3)
    out = merge_shard_results(parts)
    for i in range(len(out)):
        cands = [(int(w[i]), k) for k, (r, w, _) in enumerate(parts) if r["status"][i] == 1]
        if not cands:
            assert out[i] == parts[0][0][i]
            continue
        w, k = min(cands)
        exp = parts[k][0][i].copy()
        exp["db_seq"] += parts[k][2]
        assert out[i] == exp
    st = np.arange(0, 10_000, 100, dtype=np.uint64)
    rngs = [db_shard_records(st, 10_000, r, 4) for r in range(4)]
    assert rngs[0][1] == 100 and rngs[-1][0] == 0                  # rank 0 = top records
    assert all(rngs[r][0] == rngs[r + 1][1] for r in range(3))


def _merge_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from imsame_amd.dist import merge_db_sharded
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    r, w, lo = _fake_parts(world)[rank]
    np.save(os.path.join(out_dir, f"m{rank}.npy"), merge_db_sharded(r, w, lo, rank, world))
    dist.barrier()
    dist.destroy_process_group()


def test_db_shard_merge_over_gloo(tmp_path):
    """The collective form (min all-reduce of keys, sum all-reduce of the
    winning rows) equals the host merge on every rank."""
    from imsame_amd.dist import merge_shard_results
    world = 2
    mp.spawn(_merge_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    exp = merge_shard_results(_fake_parts(world))
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"m{r}.npy"), exp)


def _fake_kfd(tmp_path, nodes):
    """A KFD topology tree: nodes = [(simd_count, render_minor, unique_id)]
    and /dev/dri render nodes for the minors given (None: node not openable)."""
    root, dri = tmp_path / "nodes", tmp_path / "dri"
    root.mkdir()
    dri.mkdir()
    for k, (simd, minor, uid) in enumerate(nodes):
        d = root / str(k)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simd}\ndrm_render_minor {minor or 0}\n"
                                      f"unique_id {uid}\n")
        if simd and minor is not None:
            (dri / f"renderD{minor}").write_text("")
    return str(root), str(dri)


def test_visible_gpus_from_kfd_topology(tmp_path):
    """bench.py's rank launcher counts GPUs from the KFD topology, never
    through torch or HIP (a parent that starts the runtime must not fork
    children): CPU nodes and render nodes this process cannot open do not
    count; ROCR_VISIBLE_DEVICES (ordinals or GPU-<hex uuid>) applies first,
    HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES index what it leaves; a list
    stops at its first entry naming no device."""
    from imsame_amd.dist import visible_gpus, host_threads_per_rank
    nodes, dri = _fake_kfd(tmp_path, [(0, None, 0), (304, 128, 1001), (304, 129, 1002), (304, 130, 1003),
                                      (304, None, 1004)])
    vg = lambda env: visible_gpus(env, nodes, dri)            # noqa: E731
    assert vg({}) == 3                                        # the CPU node and the unopenable GPU do not count
    assert vg({"HIP_VISIBLE_DEVICES": "1"}) == 1
    assert vg({"HIP_VISIBLE_DEVICES": "0,2"}) == 2
    assert vg({"HIP_VISIBLE_DEVICES": "0,7,1"}) == 1          # stops at the first bad ordinal
    assert vg({"HIP_VISIBLE_DEVICES": "1,1"}) == 1            # a repeat ends the list
    assert vg({"CUDA_VISIBLE_DEVICES": "0,1"}) == 2
    assert vg({"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": "0,1"}) == 0   # HIP's wins, empty hides all
    assert vg({"ROCR_VISIBLE_DEVICES": "2"}) == 1
    assert vg({"ROCR_VISIBLE_DEVICES": "GPU-%x,GPU-%016x" % (1003, 1001)}) == 2
    assert vg({"ROCR_VISIBLE_DEVICES": "2,0", "HIP_VISIBLE_DEVICES": "1"}) == 1
    assert vg({"ROCR_VISIBLE_DEVICES": "2", "HIP_VISIBLE_DEVICES": "1"}) == 0
    assert visible_gpus({}, str(tmp_path / "absent"), dri) == 0
    assert host_threads_per_rank(16, 8) == 2 and host_threads_per_rank(16, 1) == 16
    assert host_threads_per_rank(4, 8) == 2 and host_threads_per_rank(128, 8) == 16


def test_visible_gpus_starts_no_runtime(tmp_path):
    """In a fresh interpreter, counting imports neither torch nor a HIP
    runtime (checked on the GPU box against torch.cuda.device_count() by
    tests/test_gpu.py:test_device_count_without_hip)."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import json, sys; sys.path.insert(0, %r); from imsame_amd.dist import visible_gpus; n = visible_gpus(); "
            "print(json.dumps({'n': n, 'hip': 'libamdhip64' in open('/proc/self/maps').read(), "
            "'torch': 'torch' in sys.modules}))" % repo)
    p = subprocess.run([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert p.returncode == 0, p.stderr.decode(errors="replace")
    got = json.loads(p.stdout.decode().strip().splitlines()[-1])
    assert not got["hip"] and not got["torch"], got
