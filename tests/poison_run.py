"""A small alignment with IMSAME_DEBUG_POISON=1 set before the library loads
(its flag is read once per process), checked against the oracle.

    IMSAME_DEBUG_POISON=1 python -m tests.poison_run   -> one JSON line on stdout

Run as a subprocess by tests/test_gpu.py::test_poison_flag_active; the
library's "[poison]" lines on stderr show the flag was live.  Test
infrastructure: it loads the oracle.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import numpy as np
    import imsame_amd
    from imsame_amd import PARITY_FIELDS
    from tests import synth
    from tests.oracle_bind import Oracle
    # 20 Mbp: random reads spend the round-1 budget (round 1b would run, but
    # is off in poison mode), 6k reads: the packed kernel's launches
    ref, rst = synth.make_reference_arr(20_000_000, 2_000, seed=81)
    q, qs = synth.make_reads_arr(ref, 6_000, 150, seed=82)
    with imsame_amd.Device(0) as dev:
        dev.index(ref, rst)
        dev.set_query(q, qs)
        res, paths, st = dev.align(n_threads=5, want_paths=True)
        res = res.copy()
    rc, exp, _ = Oracle.load().align(ref, rst, q, qs, None, 5)
    bad = [f for f in PARITY_FIELDS if not np.array_equal(res[f], exp[f])]
    print(json.dumps({"oracle_rc": rc, "mismatched_fields": bad, "reads": len(qs),
                      "accepted": int((res["status"] == 1).sum()), "n_nw": int(st.n_nw),
                      "poison": os.environ.get("IMSAME_DEBUG_POISON")}))


if __name__ == "__main__":
    main()
