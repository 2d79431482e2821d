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
