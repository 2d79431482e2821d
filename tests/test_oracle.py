"""Pin the CPU restatement (oracle/) against the reference's golden vectors.

These are the oracle's credentials: every later parity claim of the HIP path
is a comparison against this oracle (on the GPU box, where /root/reference
does not exist) or against the same golden vectors.
"""
import os
import subprocess
import tempfile

import numpy as np
import pytest

from tests import golden_io as G
from imsame_amd import fasta, PARITY_FIELDS
from tests.oracle_bind import Oracle


def test_nw_pairs_match_reference(oracle):
    rows = G.nw_pairs()
    assert len(rows) > 300
    import hashlib
    for r in rows:
        o = oracle.nw(r["X"], r["Y"], r["igap"], r["egap"])
        for k in ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y"):
            assert o[k] == r[k], (k, o[k], r[k], len(r["X"]), len(r["Y"]))
        assert len(o["text"]) == r["text_len"]
        assert hashlib.sha1(o["text"]).hexdigest() == r["text_sha1"]
        if "text" in r:
            assert o["text"].decode() == r["text"]


def test_ungapped_match_reference(oracle):
    import ctypes
    from tests.oracle_bind import UgOut
    fmt = oracle.lib.or_fmt_ld
    off = UgOut.e_value.offset
    rows, cases = G.ungapped_rows()
    assert len(rows) > 1000
    arrs = {c: (G.seqs_arrays(v["db"]), G.seqs_arrays(v["reads"])) for c, v in cases.items()}
    for r in rows:
        (db, dbs), (q, qs) = arrs[r["case"]]
        o = oracle.ungapped(db, dbs, q, qs, r["pos_db"], r["pos_q"], r["read"], r["dbseq"])
        assert (o.x_start, o.y_start, o.t_len) == (r["x_start"], r["y_start"], r["t_len"])
        buf = ctypes.create_string_buffer(64)
        # compare the full 80-bit value through the same printf as the reference driver
        fmt(ctypes.c_void_p(ctypes.addressof(o) + off), buf, 64)
        assert buf.value.decode() == r["e_hex"], (buf.value, r["e_hex"])


@pytest.mark.parametrize("name", G.e2e_cases())
def test_cli_e2e_match_reference(oracle, name):
    case = G.e2e_case(name)
    extra = case["meta"]["extra"]
    for T in case["meta"]["runs"]:
        with tempfile.TemporaryDirectory() as td:
            outp = os.path.join(td, "o.align")
            p = Oracle.run_cli(["-query", case["query"], "-db", case["db"], "-out", outp,
                                "-n_threads", T, *extra])
            blob = open(outp, "rb").read() if os.path.exists(outp) else b""
            G.check_cli_against_golden(case, int(T), p.returncode, p.stdout, blob)


def test_revcomp_match_reference(oracle):
    d = os.path.join(G.GOLDEN, "revcomp")
    names = sorted(f[:-3] for f in os.listdir(d) if f.endswith(".in"))
    assert len(names) >= 6
    for n in names:
        data = open(os.path.join(d, n + ".in"), "rb").read()
        exp = open(os.path.join(d, n + ".out"), "rb").read()
        assert oracle.revcomp(data) == exp, n


REF_BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "IMSAME")


@pytest.mark.skipif(not os.access(REF_BIN, os.X_OK), reason="oracle/_ref not built (needs /root/reference)")
def test_bench_reference_baseline_leg(oracle):
    """bench.py's CPU baseline runs the compiled reference on FASTA files of
    the sample: its accepted count equals the oracle's on the same input and
    the alignment-phase time it derives is positive and below the wall."""
    import bench
    from tests import synth
    ref, rst = synth.make_reference_arr(2_000_000, 2_000, seed=5)
    q, qs = synth.make_reads_arr(ref, 1_500, 150, seed=6)
    r = bench.run_reference(REF_BIN, ref, rst, q, qs, 3)
    rc, exp, _ = oracle.align(ref, rst, q, qs, None, 3)
    assert rc == 0
    assert r["accepted"] == int((exp["status"] == 1).sum())
    assert 0 < r["align_s"] < r["wall_s"]


def test_parallel_index_build_matches_serial(oracle, monkeypatch):
    """The oracle's index build splits the database by record ranges above
    4 Mbases (count, per-range cursors, descending scatter): every bucket must
    keep the serial build's descending-position order, so per-read results
    (which depend on the visiting order) are identical for 1 and 7 threads."""
    from tests import synth
    ref, rst = synth.make_reference_arr(6_000_000, 1_000, seed=8)
    q, qs = synth.make_reads_arr(ref, 3_000, 150, seed=9)
    out = {}
    for t in ("1", "7"):
        monkeypatch.setenv("OR_INDEX_THREADS", t)
        rc, out[t], _ = oracle.align(ref, rst, q, qs, None, 2)
        assert rc == 0
    assert (out["1"]["status"] == 1).sum() > 2_500
    assert np.array_equal(out["1"], out["7"])


@pytest.mark.parametrize("name", ["empty_not_head", "borrowed", "edges", "small_c2like"])
def test_oracle_windows_equal_whole_run(oracle, name):
    """or_align_windows (reads [a, b) of the whole query, its chunk heads) ==
    the same reads of or_align over everything: the checker used for windows
    deep inside large GPU runs (tests/test_gpu.py)."""
    case = G.e2e_case(name)
    db, dbs, brk = fasta.load(case["db"], True)
    q, qs, _ = fasta.load(case["query"])
    n = len(qs)
    runs = [int(t) for t in case["meta"]["runs"]]
    for T in sorted({runs[0], runs[-1]}):
        rc, exp, er = oracle.align(db, dbs, q, qs, None, T, brk)
        if rc:
            continue
        # one window per call, then disjoint windows in one call
        calls = [[(0, max(1, n // 2))], [(n // 3, n)], [(1, n - 1)], [(0, n // 3), (n // 2, n // 2 + 1)]]
        for ws in calls:
            ws = [w for w in ws if w[1] > w[0]]
            rc2, got, _ = oracle.align_windows(db, dbs, q, qs, ws, None, T, brk)
            assert rc2 == 0
            for (a, b), g in zip(ws, got):
                for f in PARITY_FIELDS:
                    assert np.array_equal(g[f], exp[f][a:b]), (name, T, a, b, f)
