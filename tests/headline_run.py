"""The headline benchmark's execution mode, checked against the oracle.

bench.py's C2 step -- ONE query of 1M x 150 bp reads vs the 50 Mbp reference
(BASELINE.json configs[1], bench.py's seeds), page-locked query uploaded
asynchronously, -n_threads 16, GPU_MAX_HW_QUEUES=8 set before HIP starts so
the call runs 4 lanes, two streams each, on 8 hardware queues -- then read-for-read parity
with the oracle on the start, middle (a chunk head) and end windows.

    python -m tests.headline_run        -> one JSON line on stdout
    python -m tests.headline_run --all  -> ... with EVERY one of the 1M rows
                                           compared (the oracle on the host's
                                           usable CPUs, ~2 min at 16)

Run as a subprocess by tests/test_gpu.py::test_headline_mode_parity (the
pytest process's HIP runtime has already read its own GPU_MAX_HW_QUEUES).
Test infrastructure: it loads the oracle.
"""
import json
import os
import sys
import time

if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:      # before anything starts HIP
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import imsame_amd
    from tests import parity, synth
    from tests.oracle_bind import Oracle
    t0 = time.time()
    ref, rst = synth.make_reference_arr(50_000_000, 2_000, seed=42)
    q, qs = synth.make_reads_arr(ref, 1_000_000, 150, seed=43)
    with imsame_amd.Device(0) as dev:
        dev.index(ref, rst)
        pin = imsame_amd.PinnedArray(len(q))
        pin.array[:] = q
        dev.set_query(pin.array, qs, wait=False)                  # bench.py's upload (async, in parts)
        res, _, st = dev.align(n_threads=16)
        res = res.copy()
        pin.free()
    if "--all" in sys.argv:
        # every row: 4 oracle calls of one thread per -n_threads chunk, a
        # progress line on stderr after each (a run of ~2 min that prints)
        def progress(k, n, tot):
            print(f"[headline_run] oracle part {k}/{n}: {tot['identical']}/{tot['reads_compared']} identical, "
                  f"{time.time() - t0:.0f} s", file=sys.stderr, flush=True)
        out = parity.check_all(Oracle.load(), ref, rst, q, qs, res, 16, parts=4, progress=progress)
    else:
        out = parity.check_windows(Oracle.load(), ref, rst, q, qs, res, 0, parity.windows(0, len(qs), len(qs), 16),
                                   16)
    out.update({"lanes": int(st.lanes), "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                "reads": len(qs), "accepted": int((res["status"] == 1).sum()), "n_nw": int(st.n_nw),
                "ms_align": round(st.ms_total, 3), "wall_s": round(time.time() - t0, 1)})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
