"""A world-size-1 RCCL ("nccl") process group in the same process as the
library's streams: the collectives bench.py and imsame_amd.dist run in an
N-GPU job (the counter all-reduce that replaces IMSAME's post-join sum,
IMSAME.c:460-467, and the database-shard merge), on GPU tensors, after and
between imsame_dev_align calls on cuda:0.

Run as a subprocess by tests/test_gpu.py::test_rccl_world1_next_to_library
(a fresh process: the process group, torch's HIP runtime and the library's
lanes start together).  Prints one JSON line.
"""
import json
import os
import socket
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    import imsame_amd
    from imsame_amd import PARITY_FIELDS
    from imsame_amd.dist import all_reduce, merge_db_sharded, hip_runtimes
    from tests import synth

    ref, rst = synth.make_reference_arr(3_000_000, 2_000, seed=31)
    q, qs = synth.make_reads_arr(ref, 20_000, 150, seed=32)
    out = {"backend": dist.get_backend(), "hip_runtime": hip_runtimes()}
    with imsame_amd.Device(0) as dev:
        dev.index(ref, rst)
        dev.set_query(q, qs)
        whole, _, _ = dev.align(n_threads=4)
        # the database-shard form (one shard = the whole database) and its merge
        res, win, _ = dev.align_windows(len(ref), n_threads=4)
        merged = merge_db_sharded(res, win, 0, 0, 1)
        # a collective while the library's lanes are idle, then another call
        acc = int((whole["status"] == 1).sum())
        red = all_reduce([acc, len(qs)])
        mx = all_reduce([1.5], op="max")
        again, _, _ = dev.align(n_threads=4)
    out["merge_equal"] = bool(all(np.array_equal(merged[f], whole[f]) for f in PARITY_FIELDS))
    out["rerun_equal"] = bool(all(np.array_equal(again[f], whole[f]) for f in PARITY_FIELDS))
    out["all_reduce"] = red
    out["all_reduce_max"] = mx
    out["accepted"] = acc
    out["reads"] = len(qs)
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
