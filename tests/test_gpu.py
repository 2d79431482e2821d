"""GPU parity tests: the compiled HIP path (through the C-ABI) against the
oracle and the reference's golden vectors.  Run with `pytest -m gpu`."""
import collections
import hashlib
import os
import subprocess
import tempfile

import numpy as np
import pytest

from imsame_amd import Device, render, fasta, CLI, PARITY_FIELDS, FLAG_NW32, FLAG_NW16, FLAG_NW16_ONEPASS
from imsame_amd import abi
from tests import golden_io as G
from tests import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = Device(0)
    yield d
    d.close()


def _cmp(r_dev, r_ref, limit=None):
    n = len(r_ref) if limit is None else limit
    bad = []
    for f in PARITY_FIELDS:
        idx = np.flatnonzero(r_dev[f][:n] != r_ref[f][:n])
        bad += [(int(i), f, int(r_dev[f][i]), int(r_ref[f][i])) for i in idx[:5]]
    return bad


@pytest.mark.parametrize("flags,cols", [(0, None), (FLAG_NW32, None), (0, "3"), (0, "5")],
                         ids=["auto", "nw32", "k3", "k5"])
def test_nw_pairs_match_reference_golden(dev, oracle, flags, cols, monkeypatch):
    """auto: short reads (one strip) take the packed-pair int16 kernel where
    the launch fits it; nw32: the int32 kernel for everything; k3 / k5: the
    packed kernel's 3- / 5-column latency forms forced (IMSAME_NW_K) where
    they apply (3 columns: reads <= 150 bases)."""
    if cols:
        monkeypatch.setenv("IMSAME_NW_K", cols)
    rows = G.nw_pairs()
    groups = collections.defaultdict(list)
    for r in rows:
        groups[(r["igap"], r["egap"], len(r["Y"]) <= 160)].append(r)
    checked_text = 0
    for (ig, eg, _), rs in groups.items():
        p = dev.params(igap=ig, egap=eg, min_coverage=1e-9, min_identity=1e-9, flags=flags)
        X = [r["X"].encode() for r in rs]
        Y = [r["Y"].encode() for r in rs]
        res, paths, _ = dev.nw_pairs(X, Y, p, want_paths=True)
        for k, r in enumerate(rs):
            for f in ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y"):
                assert int(res[k][f]) == r[f], (f, k, ig, eg, len(r["X"]), len(r["Y"]))
            if res[k]["status"] == 1:
                txt, ident = render(X[k], Y[k], res[k], paths[res[k]["path_off"]:res[k]["path_off"] + res[k]["path_len"]])
                assert hashlib.sha1(txt).hexdigest() == r["text_sha1"]
                assert ident == r["identities"]
                checked_text += 1
    assert checked_text > 250


@pytest.mark.parametrize("seed,cols", [(0, None), (1, None), (2, "3")])
def test_nw_packed_pairs_random_vs_oracle(dev, oracle, seed, cols, monkeypatch):
    """Packed-pair kernel on mixed shapes: every launch mixes record lengths
    12..3000 and read lengths 12..160 (unequal halves, idle groups at the
    tail), similarity 0-100 %, gap parameters up to the int16 range limit.
    cols 3: the 3-column latency form forced, reads <= 150 bases."""
    if cols:
        monkeypatch.setenv("IMSAME_NW_K", cols)
    rng = np.random.default_rng(100 + seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    # (-5,-3) leaves the int16 range (int32 kernel); mult5: every read length a
    # multiple of NW16_K (the static-last-column variant)
    gaps = [(-5, -2, 0), (0, 0, 0), (-1, 0, 0), (-40, -2, 0), (-7, -1, 0), (-5, -3, 0), (-5, -2, 1), (-2, -1, 1)]
    for ig, eg, mult5 in gaps:
        X, Y = [], []
        for k in range(97):
            xl = int(rng.choice([12, 13, 40, 150, 700, 1999, 2000, 2001, int(rng.integers(12, 3001))]))
            if mult5:
                yl = int(rng.choice([20, 100, 150, 160, 10 * int(rng.integers(2, 17))]))
            else:
                yl = int(rng.choice([12, 31, 100, 149, 150, 151, 155, 160, int(rng.integers(12, 161))]))
            if cols == "3":
                yl = min(yl, 150)
            x = acgt[rng.integers(0, 4, xl)]
            if rng.random() < 0.7:                      # read drawn from the record, mutated
                o = int(rng.integers(0, max(1, xl - yl)))
                y = x[o:o + yl].copy()
                if len(y) < yl:
                    y = np.concatenate([y, acgt[rng.integers(0, 4, yl - len(y))]])
                mut = rng.random(yl) < rng.choice([0.0, 0.02, 0.1, 0.3])
                y[mut] = acgt[rng.integers(0, 4, int(mut.sum()))]
            else:
                y = acgt[rng.integers(0, 4, yl)]
            X.append(x.tobytes()); Y.append(y.tobytes())
        p = dev.params(igap=ig, egap=eg, min_coverage=1e-9, min_identity=1e-9)
        res, _, _ = dev.nw_pairs(X, Y, p)
        p32 = dev.params(igap=ig, egap=eg, min_coverage=1e-9, min_identity=1e-9, flags=FLAG_NW32)
        res32, _, _ = dev.nw_pairs(X, Y, p32)
        for k in range(len(X)):
            o = oracle.nw(X[k], Y[k], igap=ig, egap=eg, text=False)
            for f in ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y"):
                assert int(res[k][f]) == int(o[f]), (f, k, ig, eg, len(X[k]), len(Y[k]))
                assert int(res32[k][f]) == int(o[f]), ("nw32", f, k, ig, eg)


def _params_for(dev, case):
    ex = case["meta"]["extra"]
    if not ex:
        return dev.params()
    a = dict(zip(ex[::2], ex[1::2]))
    return dev.params(min_e=float(a["-evalue"]), min_coverage=float(a["-coverage"]),
                      min_identity=float(a["-identity"]), igap=-int(a["-igap"]), egap=-int(a["-egap"]))


@pytest.mark.parametrize("name", G.e2e_cases())
def test_align_matches_oracle_e2e(dev, oracle, name):
    case = G.e2e_case(name)
    db, dbs, brk = fasta.load(case["db"], True)
    q, qs, _ = fasta.load(case["query"])
    dev.index(db, dbs, brk)
    dev.set_query(q, qs)
    for T in [int(t) for t in case["meta"]["runs"]]:
        po = _params_for(oracle, case)        # exact long double defaults on both sides
        rc, ref, er = oracle.align(db, dbs, q, qs, po, T, brk)
        lim = er if rc else None
        # default (small launches take the int32 kernel) and packed kernel forced
        for flags in (0, FLAG_NW16):
            p = _params_for(dev, case)
            p.flags = flags
            res, _, st = dev.align(n_threads=T, params=p, allow_too_long=True)
            assert not _cmp(res, ref, lim), (flags, _cmp(res, ref, lim))
            if rc:
                assert st.err_read == er


@pytest.mark.parametrize("name", G.e2e_cases())
def test_cli_matches_reference_golden(name):
    case = G.e2e_case(name)
    for T in case["meta"]["runs"]:
        with tempfile.TemporaryDirectory() as td:
            outp = os.path.join(td, "o.align")
            p = subprocess.run([CLI, "-query", case["query"], "-db", case["db"], "-out", outp, "-n_threads", T,
                                *case["meta"]["extra"]], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
            blob = open(outp, "rb").read() if os.path.exists(outp) else b""
            G.check_cli_against_golden(case, int(T), p.returncode, p.stdout, blob)


def test_revcomp_matches_reference_golden(dev, oracle):
    d = os.path.join(G.GOLDEN, "revcomp")
    names = sorted(f[:-3] for f in os.listdir(d) if f.endswith(".in"))
    for n in names:
        data = open(os.path.join(d, n + ".in"), "rb").read()
        assert dev.revcomp(data) == open(os.path.join(d, n + ".out"), "rb").read(), n
    rng = np.random.default_rng(5)
    alphabet = np.frombuffer(b"ACGTacgtNnUuRY*-\r\n\n\n>", dtype=np.uint8)
    for _ in range(20):
        blob = b">h\n" + alphabet[rng.integers(0, len(alphabet), int(rng.integers(0, 5000)))].tobytes()
        assert dev.revcomp(blob) == oracle.revcomp(blob)
    big = synth.to_fasta(*synth.make_reference_arr(3_000_000, 150, seed=3), "m", width=70)
    assert dev.revcomp(big) == oracle.revcomp(big)


def test_synthetic_c2_shape_vs_oracle_all_T(dev, oracle):
    """C2 shape scaled down: 2 Mbp in 2 kbp records, 12k x 150 bp reads."""
    ref, rst = synth.make_reference_arr(2_000_000, 2_000, seed=42)
    q, qs = synth.make_reads_arr(ref, 12_000, 150, seed=43)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    for T in (1, 8, 16):
        res, _, st = dev.align(n_threads=T)
        rc, exp, _ = oracle.align(ref, rst, q, qs, None, T)
        assert rc == 0
        assert not _cmp(res, exp), _cmp(res, exp)
        assert (res["status"] == 1).sum() > 10_000
    # tiny seed budgets (reads pause and resume every hit or three) and every
    # scan group size (lanes per read) change nothing
    for b, lanes in (("1", "1"), ("3", "1"), ("3", "4"), ("0", "4"), ("1", "16"), ("0", "16")):
        os.environ["IMSAME_SEED_BUDGET"] = b
        os.environ["IMSAME_SEED_L"] = lanes
        try:
            resb, _, stb = dev.align(n_threads=16)
        finally:
            del os.environ["IMSAME_SEED_BUDGET"], os.environ["IMSAME_SEED_L"]
        assert not _cmp(resb, res), (b, lanes, _cmp(resb, res))
    # the int32 kernel gives the same results as the packed-pair one, which
    # every launch uses when forced (by default launches < 3000 take int32)
    res32, _, _ = dev.align(n_threads=16, params=dev.params(flags=FLAG_NW32))
    assert not _cmp(res32, res), _cmp(res32, res)
    res16, _, _ = dev.align(n_threads=16, params=dev.params(flags=FLAG_NW16))
    assert not _cmp(res16, res), _cmp(res16, res)
    # the index's relative entry form (databases past 2^32 bases take it,
    # seed_kernel.hip:ent_pos), with one lane per read and with groups
    os.environ["IMSAME_ENT_REL"] = "1"
    try:
        dev.index(ref, rst)
        for lanes in ("1", "4"):
            os.environ["IMSAME_SEED_L"] = lanes
            try:
                resr, _, _ = dev.align(n_threads=16)
            finally:
                del os.environ["IMSAME_SEED_L"]
            assert not _cmp(resr, res), (lanes, _cmp(resr, res))
    finally:
        del os.environ["IMSAME_ENT_REL"]
        dev.index(ref, rst)
    # shards with the global chunk-head semantics equal the full run
    full, _, _ = dev.align(n_threads=8)
    parts = [dev.align(a, b, n_threads=8)[0] for a, b in ((0, 3001), (3001, 7777), (7777, 12_000))]
    assert not _cmp(np.concatenate(parts), full)
    # NW accounting (imsame_stats.nw_spec_waste): the device computes the
    # distinct (read, record) NWs of the reference's visiting order up to each
    # read's accepted one -- the oracle's count with its memo -- plus the
    # speculative candidates past it; the reference's own count (no memo)
    # repeats rejected records and is at least the distinct one
    import ctypes
    oracle.lib.or_last_nw.restype = ctypes.c_uint64
    oracle.lib.or_set_memo_rejected(1)
    try:
        oracle.align(ref, rst, q, qs, None, 16)
        distinct = int(oracle.lib.or_last_nw())
    finally:
        oracle.lib.or_set_memo_rejected(0)
    oracle.align(ref, rst, q, qs, None, 16)
    reference = int(oracle.lib.or_last_nw())
    res, _, st = dev.align(n_threads=16)
    print({"n_nw": st.n_nw, "spec_waste": st.nw_spec_waste, "oracle_distinct": distinct, "reference": reference})
    assert st.n_nw - st.nw_spec_waste == distinct and reference >= distinct


def test_nw16_two_pass_equals_one_pass(dev, oracle):
    """The packed kernel's two passes (score-only sweep + checkpoints, then a
    traceback band restored from the checkpoint above each best cell) give
    the one-pass kernel's rows AND paths; bands too small to hold a path make
    the waves redo their second sweep from row 1, with the same results."""
    ref, rst = synth.make_reference_arr(2_000_000, 2_000, seed=44)
    q, qs = synth.make_reads_arr(ref, 12_000, 150, seed=45)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    p1 = dev.params(flags=FLAG_NW16 | FLAG_NW16_ONEPASS)
    one, paths1, st1 = dev.align(n_threads=16, params=p1, want_paths=True)
    assert st1.nw_redo == 0 and (one["status"] == 1).sum() > 10_000

    def path(res, paths, k):
        return paths[res["path_off"][k]:res["path_off"][k] + res["path_len"][k]].tolist()

    # band sizes, and the first sweep's predicted traceback windows off ("nowin")
    for band in (None, "40", "0", "nowin"):
        os.environ["IMSAME_NW_WINDOW"] = "0" if band == "nowin" else "1"      # (imsame_dev.hip: on by default)
        if band not in (None, "nowin"):
            os.environ["IMSAME_NW_BAND"] = band
        try:
            two, paths2, st2 = dev.align(n_threads=16, params=dev.params(flags=FLAG_NW16), want_paths=True)
        finally:
            os.environ.pop("IMSAME_NW_BAND", None)
            os.environ.pop("IMSAME_NW_WINDOW", None)
        assert not _cmp(two, one), (band, _cmp(two, one))
        acc = np.flatnonzero(one["status"] == 1)
        assert all(path(two, paths2, k) == path(one, paths1, k) for k in acc[::7]), band
        if band == "0":
            assert st2.nw_redo > 0
        # most accepted reads are walked inside their predicted window
        assert (st2.nw_win == 0) if band == "nowin" else (st2.nw_win > 0.8 * len(acc)), (band, st2.nw_win)
    rc, exp, _ = oracle.align(ref, rst, q, qs, None, 16)
    assert rc == 0 and not _cmp(one, exp)


def test_c1_shape_vs_oracle(dev, oracle):
    """C1: 10k x 100 bp vs 1 Mbp (500 records), T = 1 (BASELINE configs[0])."""
    ref, rst = synth.make_reference_arr(1_000_000, 2_000, seed=1)
    q, qs = synth.make_reads_arr(ref, 10_000, 100, seed=2)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    res, _, _ = dev.align(n_threads=1)
    rc, exp, _ = oracle.align(ref, rst, q, qs, None, 1)
    assert not _cmp(res, exp), _cmp(res, exp)


def test_single_strip_reads_in_multi_strip_launch(dev, oracle):
    """163- and 400-column reads in one launch (multi-strip kernel): the
    one-strip reads read no seam (round 1 did, and failed when the seam
    buffer held large stale values)."""
    from tests.test_host import _strip_mix_pairs
    X, Y = _strip_mix_pairs()
    for _ in range(3):
        res, _, _ = dev.nw_pairs(X, Y, dev.params())
        for k in range(len(X)):
            o = oracle.nw(X[k], Y[k], text=False)
            for f in ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y"):
                assert int(res[k][f]) == int(o[f]), (f, k, len(Y[k]))


def test_long_reads_multi_strip(dev, oracle):
    """Reads longer than one strip (320 columns): 600-2500 bp vs 3 kbp records."""
    ref, rst = synth.make_reference_arr(300_000, 3_000, seed=9)
    rng = np.random.default_rng(10)
    reads = []
    for k in range(60):
        L = int(rng.integers(600, 2500))
        o = int(rng.integers(0, len(ref) - L))
        reads.append(ref[o:o + L].copy())
    q = np.concatenate(reads)
    qs = np.cumsum([0] + [len(r) for r in reads[:-1]]).astype(np.uint64)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    res, _, _ = dev.align(n_threads=1)
    rc, exp, _ = oracle.align(ref, rst, q, qs, None, 1)
    assert not _cmp(res, exp), _cmp(res, exp)


@pytest.mark.parametrize("band", ["default", "70"])
def test_long_two_pass_nw_vs_oracle(dev, oracle, band, monkeypatch):
    """nwl_kernel.hip: reads of 161 .. 3000 columns (1-5 strips) in its
    score-only pass and the walk over recomputed traceback bands -- every
    field and every path's .align text equal to the oracle's and to the
    one-pass int32 kernel (IMSAME_FLAG_NW32); a 70-step band makes the walks
    cross many bands."""
    from tests.test_host import _long_pairs
    if band != "default":
        monkeypatch.setenv("IMSAME_NWL_BAND", band)
    for seed, (ig, eg) in ((21, (-5, -2)), (22, (0, 0)), (23, (-7, -1))):
        X, Y = _long_pairs(seed, 24, 3001, 3001)
        p = dev.params(igap=ig, egap=eg, min_coverage=1e-9, min_identity=1e-9)
        res, paths, _ = dev.nw_pairs(X, Y, p, want_paths=True)
        res32, _, _ = dev.nw_pairs(X, Y, dev.params(igap=ig, egap=eg, min_coverage=1e-9, min_identity=1e-9,
                                                    flags=FLAG_NW32))
        assert not _cmp(res, res32), _cmp(res, res32)
        for k in range(len(X)):
            o = oracle.nw(X[k], Y[k], igap=ig, egap=eg, text=True)
            for f in ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y"):
                assert int(res[k][f]) == int(o[f]), (f, k, ig, eg, len(X[k]), len(Y[k]))
            txt, _ = render(X[k], Y[k], res[k], paths[res[k]["path_off"]:res[k]["path_off"] + res[k]["path_len"]])
            assert txt == o["text"], k


@pytest.mark.parametrize("mode", ["nwp", "nwl", "fallback"])
def test_packed_long_nw_kernels(dev, oracle, mode, monkeypatch, capfd):
    """nwp_kernel.hip (two long reads per wave, int16 halves in per-lane
    frames) against the oracle, against the int32 nwl_kernel (IMSAME_NWP=0)
    and with a 4-point spread limit (IMSAME_NWP_S=4) that sends every wave
    to the int32 fallback (nwl_cand) -- the kernel that ran and its fallback
    count read from the launch's diagnostics line."""
    from tests.test_host import _long_pairs
    monkeypatch.setenv("IMSAME_NW_PROF", "1")
    if mode == "nwl":
        monkeypatch.setenv("IMSAME_NWP", "0")
    if mode == "fallback":
        monkeypatch.setenv("IMSAME_NWP_S", "4")
    X, Y = _long_pairs(31, 25, 3001, 3001)          # odd: the last wave's B half repeats A
    p = dev.params(igap=-5, egap=-2, min_coverage=1e-9, min_identity=1e-9)
    capfd.readouterr()
    res, paths, _ = dev.nw_pairs(X, Y, p, want_paths=True)
    err = capfd.readouterr().err
    line = [l for l in err.splitlines() if l.startswith("[nwprof-long]")]
    assert line, err[-2000:]
    f = line[-1].split()
    kern, fbk = f[f.index("kernel") + 1], int(f[f.index("fallback") + 1])
    assert kern == ("nwl" if mode == "nwl" else "nwp"), line
    assert (fbk == 0) if mode == "nwp" else (fbk > 0 if mode == "fallback" else True), line
    for k in range(len(X)):
        o = oracle.nw(X[k], Y[k], igap=-5, egap=-2, text=True)
        for fld in ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y"):
            assert int(res[k][fld]) == int(o[fld]), (fld, k, len(X[k]), len(Y[k]))
        txt, _ = render(X[k], Y[k], res[k], paths[res[k]["path_off"]:res[k]["path_off"] + res[k]["path_len"]])
        assert txt == o["text"], k


def test_packed_long_nw_adversarial_near_limit(dev, oracle, monkeypatch, capfd):
    """nwp_kernel.hip's range proof is checked per 64-step block from the
    wave's actual extremes; inside a block it relies on drift
    bounds.  Pairs at the largest sizes nwp_fits admits, built to stress it
    (synth.adversarial_long_pairs), give every field of the oracle's NW -- whether
    a wave stayed packed or fell back to the int32 body (both counted) -- and
    the same rows as the int32 kernel (IMSAME_NWP=0)."""
    monkeypatch.setenv("IMSAME_NW_PROF", "1")
    X, Y = synth.adversarial_long_pairs()
    p = dev.params(igap=-5, egap=-2, min_coverage=1e-9, min_identity=1e-9, max_read_size=14_000)
    capfd.readouterr()
    res, _, _ = dev.nw_pairs(X, Y, p, want_paths=True)
    err = capfd.readouterr().err
    line = [l for l in err.splitlines() if l.startswith("[nwprof-long]")]
    assert line, err[-2000:]
    f = line[-1].split()
    kern, fbk = f[f.index("kernel") + 1], int(f[f.index("fallback") + 1])
    print(line[-1])
    assert kern == "nwp", line
    monkeypatch.setenv("IMSAME_NWP", "0")
    res32, _, _ = dev.nw_pairs(X, Y, p, want_paths=True)
    flds = ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y")
    for k in range(len(X)):
        o = oracle.nw(X[k], Y[k], igap=-5, egap=-2)
        for fld in flds:
            assert int(res[k][fld]) == int(o[fld]), (fld, k, len(X[k]), len(Y[k]), fbk)
            assert int(res32[k][fld]) == int(o[fld]), ("nwl", fld, k)


def _windows(n, w=1500, T=16):
    """start, middle (around a chunk head of -n_threads T) and end of a query"""
    rpt = n // T
    mid = (T // 2) * rpt
    return [(0, w), (mid - w // 2, mid + w // 2), (n - w, n)]


def test_full_c2_reference_properties(dev, oracle):
    """BASELINE configs[1] reference (50 Mbp, 25k records) with 100k reads at
    -n_threads 16: parity vs the oracle on three windows of the WHOLE query
    (start, a chunk head in the middle, the end -- 4,500 reads) + path
    self-consistency on all accepted reads' first 2000."""
    ref, rst = synth.make_reference_arr(50_000_000, 2_000, seed=42)
    q, qs = synth.make_reads_arr(ref, 100_000, 150, seed=43)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    res, paths, st = dev.align(n_threads=16, want_paths=True)
    # 40k reads per lane, a lane per two hardware queues (its rounds and round
    # 1b's; 4 queues on the box when unset)
    queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) or 4
    assert st.lanes == min(2, max(1, queues // 2))         # parts ran concurrently
    acc = res["status"] == 1
    assert acc.mean() > 0.85
    # every accepted path re-renders to the device's own identity count (all lanes)
    ka = np.flatnonzero(acc)
    for k in np.concatenate([ka[:1000], ka[ka >= len(qs) // 2][:1000]]):
        r = res[k]
        s = int(r["db_seq"])
        X = ref[int(rst[s]):int(rst[s + 1]) if s + 1 < len(rst) else len(ref)]
        Y = q[int(qs[k]):int(qs[k]) + int(r["ylen"])]
        _, ident = render(X.tobytes(), Y.tobytes(), r, paths[r["path_off"]:r["path_off"] + r["path_len"]])
        assert ident == r["identities"]
    wins = _windows(len(qs))
    rc, exp, _ = oracle.align_windows(ref, rst, q, qs, wins, None, 16)
    assert rc == 0
    for (a, b), e in zip(wins, exp):
        assert not _cmp(res[a:b], e), ((a, b), _cmp(res[a:b], e))
    assert sum(b - a for a, b in wins) >= 4_500


@pytest.mark.timeout(300)
def test_split_rounds_equal(dev, oracle, monkeypatch, capfd):
    """Split rounds (imsame_dev.hip:align_one): a later round's active reads
    scanned in two halves, the second on stream_b after (or beside) the
    first, each half's NW launch after its own scan.  With a low threshold
    (IMSAME_SPLIT_MIN) every later round splits: the per-read results equal
    the unsplit run's for the default halves, a 0.3 / 0.7 cut and two scans
    at once, and the default run equals the oracle on three windows.  A
    third of the reads are random (many rounds of many reads)."""
    ref, rst = synth.make_reference_arr(8_000_000, 2_000, seed=81)
    q, qs = synth.make_reads_arr(ref, 150_000, 150, seed=82, frac_true=0.67)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    # (split rounds belong to the joined rounds: with independent pipelines
    # each pipeline's rounds stay whole)
    monkeypatch.setenv("IMSAME_PIPES", "0")
    monkeypatch.setenv("IMSAME_SPLIT_ROUNDS", "0")
    base, pb, sb = dev.align(n_threads=16, want_paths=True)
    monkeypatch.delenv("IMSAME_SPLIT_ROUNDS")
    monkeypatch.setenv("IMSAME_SPLIT_MIN", "64")
    monkeypatch.setenv("IMSAME_DEBUG_ROUNDS", "1")      # split rounds print "[round k split]"
    res = None
    # (spec 2 < spec_weak 8: reads with no rejection yet emit up to 8 -- the
    # first half's list room is max(spec, spec_weak) per read)
    for env in [{}, {"IMSAME_SPLIT_FRAC": "0.3"}, {"IMSAME_SPLIT_SEQ": "0"},
                {"IMSAME_SPEC": "2", "IMSAME_SPEC_WEAK": "8"}]:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        capfd.readouterr()
        r, pp, st = dev.align(n_threads=16, want_paths=True)
        err = capfd.readouterr().err
        for k in env:
            monkeypatch.delenv(k)
        assert " split] " in err, (env, err[-1500:])
        assert not _cmp(r, base), (env, _cmp(r, base))
        assert (st.n_nw == sb.n_nw or "IMSAME_SPEC" in env) and st.rounds >= 2, (env, st.n_nw, sb.n_nw, st.rounds)
        for k in np.flatnonzero(base["status"] == 1)[::211]:
            s_ = int(base[k]["db_seq"])
            X = ref[int(rst[s_]):int(rst[s_]) + 2_000].tobytes()
            Y = q[int(qs[k]):int(qs[k]) + 150].tobytes()
            t1, _ = render(X, Y, r[k], pp[r[k]["path_off"]:r[k]["path_off"] + r[k]["path_len"]])
            t0, _ = render(X, Y, base[k], pb[base[k]["path_off"]:base[k]["path_off"] + base[k]["path_len"]])
            assert t1 == t0, (env, k)
        if res is None:
            res = r
    wins = _windows(len(qs))
    rc, exp, _ = oracle.align_windows(ref, rst, q, qs, wins, None, 16)
    assert rc == 0
    for (a, b), e in zip(wins, exp):
        assert not _cmp(res[a:b], e), ((a, b), _cmp(res[a:b], e))


@pytest.mark.timeout(900)
@pytest.mark.timeout(900)
def test_headline_mode_parity():
    """The benchmark's own execution mode: 1M x 150 bp vs the 50 Mbp C2
    reference in ONE call, async page-locked upload, -n_threads 16, with
    GPU_MAX_HW_QUEUES=8 set before HIP starts (a subprocess: this process's
    runtime keeps the box's value) -- 3 lanes, each with its rounds' and
    round 1b's stream on a hardware queue of its own -- and read-for-read
    oracle parity on ALL 1,000,000 rows (the oracle on the host's CPUs,
    ~2 min at 16; tests/parity.py:check_all)."""
    import json
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GPU_MAX_HW_QUEUES="8")
    p = subprocess.run([sys.executable, "-u", "-m", "tests.headline_run", "--all"], cwd=repo, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=840)
    assert p.returncode == 0, p.stderr[-3000:].decode(errors="replace")
    d = json.loads(p.stdout.decode().strip().splitlines()[-1])
    print(d)
    assert d["lanes"] == 3, d                  # 8 queues hold 4 lanes of two streams; LANES_DEF = 3
    assert d["reads_compared"] == 1_000_000 and d["identical"] == d["reads_compared"], d
    assert d["accepted"] > 850_000


@pytest.mark.timeout(300)
def test_poison_flag_active():
    """IMSAME_DEBUG_POISON=1: in a subprocess, so the flag is
    read at library load -- every reused device buffer is filled with poison
    on its call's stream and every kernel is followed by a named stream
    synchronize.  The "[poison]" lines show it was live; the rows stay
    oracle-exact (no kernel reads memory it did not write)."""
    import json
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, IMSAME_DEBUG_POISON="1")
    p = subprocess.run([sys.executable, "-u", "-m", "tests.poison_run"], cwd=repo, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:].decode(errors="replace")
    err = p.stderr.decode(errors="replace")
    assert err.count("[poison] nw16_kernel") > 0 and err.count("[poison] seed kernel") > 0
    d = json.loads(p.stdout.decode().strip().splitlines()[-1])
    assert d["oracle_rc"] == 0 and d["mismatched_fields"] == [] and d["accepted"] > 5000, d


@pytest.fixture
def oracle_memo(oracle):
    """The oracle with its test-speed memo of rejected (read, record) pairs
    (identical results): the reference re-runs NW for
    every e-value-passing hit, hundreds per 10 kbp read."""
    oracle.lib.or_set_memo_rejected(1)
    yield oracle
    oracle.lib.or_set_memo_rejected(0)


@pytest.mark.timeout(300)
def test_c3_reference_500mbp(dev, oracle_memo):
    """BASELINE configs[2] per-GPU shard: 1.25M x 150 bp reads (10M / 8) vs
    the 500 Mbp reference (250k records, 4 GB of CSR entries), -n_threads 16:
    oracle parity on three windows of the whole query (start, a chunk head in
    the middle, the end), path self-consistency and the accepted fraction."""
    ref, rst = synth.make_reference_arr(500_000_000, 2_000, seed=43)
    q, qs = synth.make_reads_arr(ref, 1_250_000, 150, seed=44)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    res, paths, st = dev.align(n_threads=16, want_paths=True)
    acc = res["status"] == 1
    assert acc.mean() > 0.85, acc.mean()
    for k in np.flatnonzero(acc)[:1000]:
        r = res[k]
        s = int(r["db_seq"])
        X = ref[int(rst[s]):int(rst[s + 1]) if s + 1 < len(rst) else len(ref)]
        Y = q[int(qs[k]):int(qs[k]) + int(r["ylen"])]
        _, ident = render(X.tobytes(), Y.tobytes(), r, paths[r["path_off"]:r["path_off"] + r["path_len"]])
        assert ident == r["identities"]
    wins = _windows(len(qs))
    rc, exp, _ = oracle_memo.align_windows(ref, rst, q, qs, wins, None, 16)
    assert rc == 0
    for (a, b), e in zip(wins, exp):
        assert not _cmp(res[a:b], e), ((a, b), _cmp(res[a:b], e))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("rec_bp,cap", [(2_000, 10_001), (12_000, 12_001)], ids=["c5_2kbp_records", "c5_12kbp_records"])
def test_c5_ont_long_reads_raised_cap(dev, oracle_memo, rec_bp, cap):
    """BASELINE configs[4] shape: 10 kbp ONT-like reads (5 % sub, 2.5 % ins,
    2.5 % del) with the raised MAX_READ_SIZE (SURVEY 8(c) iv).  Against the
    C5 2 kbp records every candidate is rejected (coverage len/ylen < 0.5);
    against 12 kbp records reads are accepted with 120M-cell matrices.  At
    the stock cap the first e-value pass is the fatal size error."""
    n = 16 if rec_bp == 2_000 else 10
    ref, rst = synth.make_reference_arr(rec_bp * 300, rec_bp, seed=48)
    q, qs = synth.make_long_reads_arr(ref, n, 10_000, seed=49)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    res, _, st = dev.align(n_threads=8, params=dev.params(max_read_size=cap))
    rc, exp, _ = oracle_memo.align(ref, rst, q, qs, oracle_memo.params(max_read_size=cap), 8)
    assert rc == 0
    assert not _cmp(res, exp), _cmp(res, exp)
    # 2 kbp records cannot give the 2500 identities a 10 kbp read needs: every
    # candidate is rejected a priori (seed_kernel.hip:nw_cannot_accept)
    assert (st.n_nw > 0) == (rec_bp > 10_000)
    if rec_bp > 10_000:
        assert (res["status"] == 1).sum() >= n // 2
    _, _, st3 = dev.align(n_threads=8, allow_too_long=True)
    rc3, _, er3 = oracle_memo.align(ref, rst, q, qs, None, 8)
    assert rc3 == abi.IMSAME_E_READ_TOO_LONG and st3.err_read == er3


@pytest.mark.timeout(600)
def test_wide_database_past_4_gbases(oracle_memo):
    """a 4.4 Gbase database (2.2M records of 2 kbp), past
    the 2^32 positions a u32 index holds.  Reads come from the last 150 Mbp,
    so their seeds, records and NW rows lie on both sides of 2^32.  Oracle
    parity (u64 positions) on every read; path self-consistency."""
    total = 4_400_000_000
    ref, rst = synth.make_reference_arr(total, 2_000, seed=50)
    tail = total - 150_000_000
    q, qs = synth.make_reads_arr(ref[tail:], 1_500, 150, seed=51)
    with Device(0) as d:
        d.index(ref, rst)
        d.set_query(q, qs)
        res, paths, st = d.align(n_threads=1, want_paths=True)
    acc = res["status"] == 1
    assert acc.mean() > 0.85, acc.mean()
    assert (rst[res["db_seq"][acc]] >= 2 ** 32).sum() > 500       # records past 2^32 found
    for k in np.flatnonzero(acc)[:300]:
        r = res[k]
        s = int(r["db_seq"])
        X = ref[int(rst[s]):int(rst[s + 1]) if s + 1 < len(rst) else len(ref)]
        Y = q[int(qs[k]):int(qs[k]) + int(r["ylen"])]
        _, ident = render(X.tobytes(), Y.tobytes(), r, paths[r["path_off"]:r["path_off"] + r["path_len"]])
        assert ident == r["identities"]
    rc, exp, _ = oracle_memo.align(ref, rst, q, qs, None, 1)
    assert rc == 0
    assert not _cmp(res, exp), _cmp(res, exp)


@pytest.mark.parametrize("name", G.e2e_cases())
def test_sliced_database_matches_oracle_e2e(dev, oracle, name):
    """imsame_dev_align_sliced with every record a slice of its own (the
    finest cut) on the golden end-to-end cases: k-mer reset bitmaps shifted
    into each slice, the whole database's L_DB in the e-value, every
    -n_threads.  Cases that reach the size abort are refused (IMSAME_E_ARG)."""
    case = G.e2e_case(name)
    db, dbs, brk = fasta.load(case["db"], True)
    q, qs, _ = fasta.load(case["query"])
    dev.set_query(q, qs)
    rec_len = np.diff(np.append(dbs, len(db)).astype(np.int64))
    read_len = np.diff(np.append(qs, len(q)).astype(np.int64))
    for T in [int(t) for t in case["meta"]["runs"]]:
        p = _params_for(dev, case)
        po = _params_for(oracle, case)
        if max(rec_len.max(initial=0), read_len.max(initial=0)) > p.max_read_size:
            with pytest.raises(abi_error()) as e:
                dev.align_sliced(db, dbs, 1, brk, n_threads=T, params=p)
            assert e.value.code == abi.IMSAME_E_ARG
            continue
        rc, ref, er = oracle.align(db, dbs, q, qs, po, T, brk)
        assert rc == 0
        res, _, _, ns = dev.align_sliced(db, dbs, 1, brk, n_threads=T, params=p)
        assert ns == len(dbs)
        assert not _cmp(res, ref), _cmp(res, ref)


def abi_error():
    from imsame_amd import ImsameError
    return ImsameError


@pytest.mark.parametrize("slice_bases", [1_000_000, 301_000])
def test_sliced_database_matches_whole(dev, oracle, slice_bases):
    """Memory-capped multi-pass index: a 4 Mbp database
    searched in slices gives the whole-database results bit for bit (oracle
    and single-index device pass), with paths that render to the same
    identities, for -n_threads 1 and 5."""
    ref, rst = synth.make_reference_arr(4_000_000, 2_000, seed=21)
    q, qs = synth.make_reads_arr(ref, 4_000, 150, seed=22)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    wholes = {T: dev.align(n_threads=T)[0] for T in (1, 5)}     # before the slices replace the index
    for T in (1, 5):
        whole = wholes[T]
        res, paths, st, ns = dev.align_sliced(ref, rst, slice_bases, n_threads=T, want_paths=True)
        assert ns == -(-4_000_000 // (slice_bases - slice_bases % 2_000))
        assert not _cmp(res, whole), _cmp(res, whole)
        rc, exp, _ = oracle.align(ref, rst, q, qs, None, T)
        assert rc == 0 and not _cmp(res, exp), _cmp(res, exp)
        acc = np.flatnonzero(res["status"] == 1)
        assert len(acc) > 3_400 and st.n_accepted == len(acc)
        for k in acc[:300]:
            r = res[k]
            s = int(r["db_seq"])
            X = ref[int(rst[s]):int(rst[s]) + 2_000]
            Y = q[int(qs[k]):int(qs[k]) + int(r["ylen"])]
            _, ident = render(X.tobytes(), Y.tobytes(), r, paths[r["path_off"]:r["path_off"] + r["path_len"]])
            assert ident == r["identities"]


@pytest.mark.parametrize("world", [2, 3])
def test_db_shards_min_merge_matches_whole(dev, oracle, world):
    """Database shards (one per GPU in a multi-GPU run, here one after the
    other on one device): each shard's index + imsame_dev_align_windows with
    the whole database's L_DB and no caps, merged by the smallest (window,
    shard) key (imsame_amd.dist) -- bit-exact vs the whole-database oracle."""
    from imsame_amd.dist import db_shard_records, merge_shard_results
    ref, rst = synth.make_reference_arr(3_000_000, 2_000, seed=31)
    q, qs = synth.make_reads_arr(ref, 3_000, 150, seed=32)
    dev.set_query(q, qs)
    for T in (1, 4):
        parts = []
        for rank in range(world):
            lo, hi = db_shard_records(rst, len(ref), rank, world)
            base = int(rst[lo])
            end = int(rst[hi]) if hi < len(rst) else len(ref)
            dev.index(ref[base:end], rst[lo:hi] - np.uint64(base))
            res, win, _ = dev.align_windows(len(ref), n_threads=T)
            assert (win[res["status"] == 1] != np.iinfo(np.uint64).max).all()
            parts.append((res, win, lo))
        got = merge_shard_results(parts)
        rc, exp, _ = oracle.align(ref, rst, q, qs, None, T)
        assert rc == 0 and not _cmp(got, exp), _cmp(got, exp)
        assert (got["status"] == 1).sum() > 2_500


@pytest.mark.parametrize("name", G.e2e_cases())
def test_cli_sliced_matches_reference_golden(name):
    """The CLI with -slice_bases (database indexed 3 kbp at a time) writes the
    reference's .align bytes and [INFO] lines; inputs where the size abort
    could fire are refused with a message instead."""
    case = G.e2e_case(name)
    db, dbs, _ = fasta.load(case["db"], True)
    q, qs, _ = fasta.load(case["query"])
    big = max(np.diff(np.append(dbs, len(db)).astype(np.int64)).max(initial=0),
              np.diff(np.append(qs, len(q)).astype(np.int64)).max(initial=0)) > 3000
    for T in case["meta"]["runs"]:
        with tempfile.TemporaryDirectory() as td:
            outp = os.path.join(td, "o.align")
            p = subprocess.run([CLI, "-query", case["query"], "-db", case["db"], "-out", outp, "-n_threads", T,
                                "-slice_bases", "3000", *case["meta"]["extra"]],
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
            if big:
                assert p.returncode != 0 and b"-slice_bases" in p.stdout
                continue
            blob = open(outp, "rb").read() if os.path.exists(outp) else b""
            G.check_cli_against_golden(case, int(T), p.returncode, p.stdout, blob)


def test_query_shards_equal_whole_run(dev, oracle):
    """imsame_dev_set_query_range: each device holds only its shard of the
    query (bench.py strong scaling, imsame -devices).  Shards of the
    bench's split for 2, 3 and 8 ranks, and cuts after empty-free odd
    places, concatenate to the whole-query run bit for bit (-n_threads 16:
    chunk heads inside and outside the shards)."""
    from imsame_amd.dist import shard_range
    ref, rst = synth.make_reference_arr(2_000_000, 2_000, seed=42)
    q, qs = synth.make_reads_arr(ref, 12_000, 150, seed=43)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    whole, _, _ = dev.align(n_threads=16)
    for world in (2, 3, 8):
        parts = []
        for rank in range(world):
            a, b = shard_range(len(qs), rank, world)
            dev.set_query(q, qs, a, b)
            parts.append(dev.align(a, b, n_threads=16)[0])
        got = np.concatenate(parts)
        assert not _cmp(got, whole), (world, _cmp(got, whole))
    dev.set_query(q, qs, 749, 7501)                       # sub-ranges of a shard
    got = np.concatenate([dev.align(749, 750, n_threads=16)[0], dev.align(750, 7501, n_threads=16)[0]])
    assert not _cmp(got, whole[749:7501])
    with pytest.raises(abi_error()):
        dev.align(0, 10, n_threads=16)                    # outside the uploaded range
    rc, exp, _ = oracle.align(ref, rst, q, qs, None, 16)
    assert rc == 0 and not _cmp(whole, exp)


def test_async_query_upload_equals_sync(dev, monkeypatch):
    """imsame_dev_set_query_range_async: the copies are queued in parts and
    each lane of the next align waits only for the parts holding its reads
    (bench.py's step).  4 lanes over a page-locked query give the rows of
    the waited upload; a second queued upload (another shard) replaces the
    first before any align; imsame_dev_sync waits without an align."""
    import imsame_amd
    ref, rst = synth.make_reference_arr(2_000_000, 2_000, seed=52)
    q, qs = synth.make_reads_arr(ref, 140_000, 150, seed=53)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    whole, _, st0 = dev.align(n_threads=16)
    pin = imsame_amd.PinnedArray(len(q))
    pin.array[:] = q
    monkeypatch.setenv("IMSAME_LANES", "4")
    dev.set_query(pin.array, qs, wait=False)
    got, _, st = dev.align(n_threads=16)
    assert st.lanes == 4 and not _cmp(got, whole)
    dev.set_query(pin.array, qs, 0, 70_000, wait=False)
    dev.set_query(pin.array, qs, 70_000, 140_000, wait=False)
    got, _, st = dev.align(n_threads=16)
    assert st.lanes == 2 and not _cmp(got, whole[70_000:])
    dev.set_query(pin.array, qs, 1, 139_999, wait=False)
    dev.sync()
    got, _, _ = dev.align(n_threads=16)
    assert not _cmp(got, whole[1:139_999])
    pin.free()


def test_path_arena_overflow_rewalks_only_lost_reads(dev, monkeypatch):
    """A device path arena too small for the accepted reads' paths: only the
    reads whose path did not fit are re-walked (NW is pure, Appendix A Q18),
    giving the same rows and the same .align text as an arena with room;
    a host arena too small gets IMSAME_E_PATHS and fetches afterwards."""
    ref, rst = synth.make_reference_arr(2_000_000, 2_000, seed=7)
    q, qs = synth.make_reads_arr(ref, 6_000, 150, seed=8, ins=0.01, dele=0.01)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    base, bp, bst = dev.align(n_threads=8, want_paths=True)
    assert bst.n_rewalk == 0
    monkeypatch.setenv("IMSAME_DEV_PATHS_CAP", "3000")
    res, paths, st = dev.align(n_threads=8, want_paths=True, paths_cap=16)
    monkeypatch.delenv("IMSAME_DEV_PATHS_CAP")
    assert st.n_rewalk > 100, st.n_rewalk
    assert not _cmp(res, base)
    for k in np.flatnonzero(res["status"] == 1)[::7]:
        r, r0 = res[k], base[k]
        s = int(r["db_seq"])
        X = ref[int(rst[s]):int(rst[s]) + 2_000].tobytes()
        Y = q[int(qs[k]):int(qs[k]) + 150].tobytes()
        t1, _ = render(X, Y, r, paths[r["path_off"]:r["path_off"] + r["path_len"]])
        t0, _ = render(X, Y, r0, bp[r0["path_off"]:r0["path_off"] + r0["path_len"]])
        assert t1 == t0, k


@pytest.mark.parametrize("name", G.e2e_cases())
def test_cli_devices_matches_reference_golden(name):
    """imsame -devices 0,0 (two contexts, each holding one shard of the
    query) with tiny batches and 3 render threads: the reference's .align
    bytes and [INFO] lines for every -n_threads."""
    case = G.e2e_case(name)
    for T in case["meta"]["runs"]:
        with tempfile.TemporaryDirectory() as td:
            outp = os.path.join(td, "o.align")
            p = subprocess.run([CLI, "-query", case["query"], "-db", case["db"], "-out", outp, "-n_threads", T,
                                "-devices", "0,0", "-batch_reads", "7", "-render_threads", "3",
                                *case["meta"]["extra"]], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
            blob = open(outp, "rb").read() if os.path.exists(outp) else b""
            G.check_cli_against_golden(case, int(T), p.returncode, p.stdout, blob)


def test_cli_multi_device_output_identical(tmp_path):
    """C2 shape (2 Mbp, 12k reads) through the CLI: one context vs three
    (-devices 0,0,0) with batches of 1000 reads, one render thread, 4
    lanes handing over their parts out of order, and 3 lanes of 2 pieces each
    -- identical .align bytes."""
    ref, rst = synth.make_reference_arr(2_000_000, 2_000, seed=42)
    q, qs = synth.make_reads_arr(ref, 12_000, 150, seed=43)
    dbf, qf = str(tmp_path / "db.fa"), str(tmp_path / "q.fa")
    synth.write_fasta(dbf, ref, rst, "ref")
    synth.write_fasta(qf, q, qs, "read", width=0)
    outs = []
    for extra, env in (([], {}), (["-devices", "0,0,0", "-batch_reads", "1000"], {}), (["-render_threads", "1"], {}),
                       ([], {"IMSAME_LANES": "4", "IMSAME_LANE_MIN": "1000"}),
                       ([], {"IMSAME_LANES": "3", "IMSAME_LANE_PARTS": "2", "IMSAME_LANE_MIN": "1000"})):
        o = str(tmp_path / f"o{len(outs)}.align")
        p = subprocess.run([CLI, "-query", qf, "-db", dbf, "-out", o, "-n_threads", "16", *extra],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300, env=dict(os.environ, **env))
        assert p.returncode == 0, p.stderr[-2000:]
        assert b'"accepted"' in p.stderr
        outs.append(open(o, "rb").read())
    assert all(o == outs[0] for o in outs[1:])
    assert outs[0].count(b" $$$$$$$ \n") > 10_000


@pytest.mark.timeout(900)
@pytest.mark.parametrize("rec_bp,cap", [(2_000, 10_001), (12_001, 12_001)], ids=["c5_2kbp", "c5w_12kbp"])
def test_c5_full_50mbp_database(dev, oracle_memo, rec_bp, cap):
    """BASELINE configs[4] at its real database size (50 Mbp, so the e-value
    tables use C5's L_DB): 6 ONT-like 10 kbp reads vs 2 kbp records (every
    read rejected a priori: no record can hold the identities a 10 kbp read
    needs, seed_kernel.hip:read_irrelevant) and vs 12 kbp records (the
    long-read NW runs, 120M cells per candidate) -- every field equal to the
    oracle's, which runs the reference's full scan and NWs."""
    ref, rst = synth.make_reference_arr(50_004_000 if rec_bp > 10_000 else 50_000_000, rec_bp, seed=42)
    q, qs = synth.make_long_reads_arr(ref, 6, 10_000, seed=48)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    res, _, st = dev.align(n_threads=3, params=dev.params(max_read_size=cap))
    rc, exp, _ = oracle_memo.align(ref, rst, q, qs, oracle_memo.params(max_read_size=cap), 3)
    assert rc == 0
    assert not _cmp(res, exp), _cmp(res, exp)
    if rec_bp > 10_000:
        assert st.n_nw > 0 and (res["status"] == 1).sum() >= 3
        # the packed long-read kernel ran every long launch, none fell back
        assert st.launch_nwp != 0 and st.nw_fallback == 0, (hex(st.launch_nwp), st.nw_fallback)
    else:
        assert st.n_nw == 0 and st.n_hits == 0 and (res["status"] == 1).sum() == 0


def test_eight_skewed_lanes_equal_one_lane(dev, monkeypatch):
    """8 lanes (the default from 1M reads) cut with skewed shares (weights
    0.6 .. 1.4, imsame_dev_align) on their own hardware queues: the same rows
    as one lane, and the same rows at skew 0.9 (the smallest lane 1/8 of the
    average)."""
    ref, rst = synth.make_reference_arr(3_000_000, 2_000, seed=71)
    q, qs = synth.make_reads_arr(ref, 320_000, 150, seed=72)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    monkeypatch.setenv("IMSAME_LANES", "1")
    one, _, s1 = dev.align(n_threads=16)
    monkeypatch.setenv("IMSAME_LANES", "8")
    eight, _, s8 = dev.align(n_threads=16)
    assert s1.lanes == 1 and s8.lanes == 8
    assert not _cmp(eight, one), _cmp(eight, one)
    monkeypatch.setenv("IMSAME_LANE_SKEW", "0.9")
    sk, _, _ = dev.align(n_threads=16)
    assert not _cmp(sk, one), _cmp(sk, one)


def test_align_parts_hand_over_every_lane(dev, monkeypatch):
    """imsame_dev_align_parts: the lanes' parts cover the range exactly, each
    with its own paths, and give the rows and .align text of one call to
    imsame_dev_align (the CLI renders parts as they arrive)."""
    ref, rst = synth.make_reference_arr(4_000_000, 2_000, seed=61)
    q, qs = synth.make_reads_arr(ref, 140_000, 150, seed=62, ins=0.003, dele=0.003)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    whole, pw, _ = dev.align(n_threads=7, want_paths=True)
    monkeypatch.setenv("IMSAME_LANE_MIN", "1000")
    for lanes, pieces in (("1", "1"), ("4", "1"), ("3", "3")):
        monkeypatch.setenv("IMSAME_LANES", lanes)
        monkeypatch.setenv("IMSAME_LANE_PARTS", pieces)       # pieces per lane, handed over in turn
        res, parts, st = dev.align_parts(n_threads=7, want_paths=True)
        assert st.lanes == int(lanes) and len(parts) == int(lanes) * int(pieces)
        assert st.n_reads == len(qs)
        cov = sorted((a, b) for a, b, *_ in parts)
        assert cov[0][0] == 0 and cov[-1][1] == len(qs) and all(x[1] == y[0] for x, y in zip(cov, cov[1:]))
        assert all(s == 0 and e == 2 ** 64 - 1 for _, _, s, e, _ in parts)
        assert not _cmp(res, whole)
        for a, b, _, _, pp in parts:
            for k in np.flatnonzero(res["status"][a:b] == 1)[::97] + a:
                r, r0 = res[k], whole[k]
                s_ = int(r["db_seq"])
                X = ref[int(rst[s_]):int(rst[s_]) + 2_000].tobytes()
                Y = q[int(qs[k]):int(qs[k]) + 150].tobytes()
                t1, _ = render(X, Y, r, pp[r["path_off"]:r["path_off"] + r["path_len"]])
                t0, _ = render(X, Y, r0, pw[r0["path_off"]:r0["path_off"] + r0["path_len"]])
                assert t1 == t0, k


@pytest.mark.timeout(300)
def test_nw16_launch_forms_equal(dev, oracle, monkeypatch):
    """nw16_kernel's launch forms on a 1/8-shard-sized call (3 lanes):
    10 or 5 columns per lane (imsame_dev.hip:nw16_k) and persistent or
    non-persistent launches (one wave per task, arena slots from a per-XCD
    free bitmap, nw16_kernel.hip:nw_slot_claim).  Every per-read field and
    every accepted path's text equal across the forms, and the default run
    equals the oracle on three windows."""
    ref, rst = synth.make_reference_arr(4_000_000, 2_000, seed=71)
    q, qs = synth.make_reads_arr(ref, 125_000, 150, seed=72, ins=0.003, dele=0.003)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    base, pb, sb = dev.align(n_threads=16, want_paths=True)
    assert sb.launch_np != 0                      # the XCC probe passed: non-persistent launches ran
    runs = {}
    for name, env in [("k10_persistent", {"IMSAME_NW_K": "10", "IMSAME_NW_PERSIST": "1"}),
                      ("k5_all", {"IMSAME_NW_K": "5"}),
                      ("k3_all", {"IMSAME_NW_K": "3"}),
                      ("k10_np", {"IMSAME_NW_K": "10"})]:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        runs[name] = dev.align(n_threads=16, want_paths=True)
        for k in env:
            monkeypatch.delenv(k)
    st = runs["k10_persistent"][2]
    assert st.launch_np == 0 and st.launch_k5 == 0
    st = runs["k5_all"][2]
    assert st.launch_k5 == st.launch_pk and st.launch_pk != 0
    st = runs["k3_all"][2]        # the 3-column latency form (reads <= 150 bases; longer: 5 columns)
    assert st.launch_k3 != 0 and (st.launch_k3 | st.launch_k5) == st.launch_pk, (hex(st.launch_k3), hex(st.launch_pk))
    for name, (res, pp, st) in runs.items():
        assert not _cmp(res, base), (name, _cmp(res, base))
        if st.launch_np:                          # round 1b ran in both (its speculation sets n_nw)
            assert st.n_nw == sb.n_nw
        for k in np.flatnonzero(base["status"] == 1)[::97]:
            r, r0 = res[k], base[k]
            s_ = int(r0["db_seq"])
            X = ref[int(rst[s_]):int(rst[s_]) + 2_000].tobytes()
            Y = q[int(qs[k]):int(qs[k]) + 150].tobytes()
            t1, _ = render(X, Y, r, pp[r["path_off"]:r["path_off"] + r["path_len"]])
            t0, _ = render(X, Y, r0, pb[r0["path_off"]:r0["path_off"] + r0["path_len"]])
            assert t1 == t0, (name, k)
    wins = _windows(len(qs))
    rc, exp, _ = oracle.align_windows(ref, rst, q, qs, wins, None, 16)
    assert rc == 0
    for (a, b), e in zip(wins, exp):
        assert not _cmp(base[a:b], e), ((a, b), _cmp(base[a:b], e))


def test_lanes_equal_one_lane(dev, monkeypatch):
    """Three concurrent lanes (parts of a call on three streams) against one
    lane: identical per-read rows and identical .align text for every
    accepted read (each lane's paths follow the previous lanes' in the
    arena).  The same seed budget schedule in both (by default a lane of
    < 100k reads grows its budget faster, which reshapes the work only)."""
    ref, rst = synth.make_reference_arr(4_000_000, 2_000, seed=61)
    q, qs = synth.make_reads_arr(ref, 140_000, 150, seed=62, ins=0.003, dele=0.003)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    monkeypatch.setenv("IMSAME_LANES", "3")                  # 3 whatever the box's queues
    monkeypatch.setenv("IMSAME_SEED_GROW", "8")
    two, p2, s2 = dev.align(n_threads=7, want_paths=True, paths_cap=64)     # small host arena: fetch path
    monkeypatch.setenv("IMSAME_LANES", "1")
    one, p1, s1 = dev.align(n_threads=7, want_paths=True)
    monkeypatch.delenv("IMSAME_LANES")
    assert s2.lanes == 3 and s1.lanes == 1
    assert not _cmp(two, one)
    assert s2.n_nw == s1.n_nw and s2.n_accepted == s1.n_accepted and s2.ms_nw_busy > 0
    for k in np.flatnonzero(two["status"] == 1)[::53]:
        r2, r1 = two[k], one[k]
        s = int(r2["db_seq"])
        X = ref[int(rst[s]):int(rst[s]) + 2_000].tobytes()
        Y = q[int(qs[k]):int(qs[k]) + 150].tobytes()
        t2, _ = render(X, Y, r2, p2[r2["path_off"]:r2["path_off"] + r2["path_len"]])
        t1, _ = render(X, Y, r1, p1[r1["path_off"]:r1["path_off"] + r1["path_len"]])
        assert t2 == t1, k


def test_short_call_without_shared_arena(oracle, monkeypatch):
    """When the shared non-persistent NW arena cannot be allocated (free HBM
    short of it: e.g. after a long-read call grew the context's persistent
    traceback arena to most of HBM; IMSAME_DEBUG_NP_SKIP simulates it), every
    launch must be PLANNED persistent (plan_nw checks the arena the context
    holds), and round 1b's two concurrent launches must not both fall back to
    the one persistent arena (they shared its slots).  Rows equal
    the oracle's; the same call with the arena runs non-persistent launches."""
    ref, rst = synth.make_reference_arr(2_000_000, 2_000, seed=42)
    q, qs = synth.make_reads_arr(ref, 12_000, 150, seed=43)
    rc, exp, _ = oracle.align(ref, rst, q, qs, None, 16)
    assert rc == 0
    for skip in ("1", "0"):
        monkeypatch.setenv("IMSAME_DEBUG_NP_SKIP", skip)
        with Device(0) as d:
            d.index(ref, rst)
            d.set_query(q, qs)
            res, _, st = d.align(n_threads=16)
        assert not _cmp(res, exp), (skip, _cmp(res, exp))
        if skip == "1":
            assert st.launch_np == 0, hex(st.launch_np)   # no shared arena: every launch persistent
        else:
            assert st.launch_np != 0                      # (the box has the XCD probe: np launches)


def test_bench_launches_ranks_itself():
    """`bench.py --gpus 2` with no launcher starts its two ranks itself (the
    driver's form of the N-GPU run), here as a gloo rehearsal on one card: the
    line says n_gpus 2, and the shards' accepted reads sum to a one-rank run's.
    Two forms: the fixed `--device 0` rehearsal, and the driver's own form
    without --device -- the launcher counts the GPUs without HIP (KFD
    topology) and, told that 2 are visible, maps rank r onto card r mod the
    real count."""
    import json
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    base = [sys.executable, "-u", "bench.py", "--steps", "1", "--warmup", "0", "--cpu-sample", "0", "--e2e", "off",
            "--reads", "100000"]
    lines = {}
    for key, extra in (("dev0", ["--gpus", "2", "--dist-backend", "gloo", "--device", "0"]),
                       ("nodev", ["--gpus", "2", "--dist-backend", "gloo", "--device-count-override", "2"]),
                       ("one", ["--gpus", "1"])):
        p = subprocess.run(base + extra, cwd=repo, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           timeout=900)
        assert p.returncode == 0, p.stderr[-3000:].decode(errors="replace")
        lines[key] = json.loads([x for x in p.stdout.decode().splitlines() if x.startswith("{")][-1])
    one = lines["one"]
    print(json.dumps({k: {f: lines[k][f] for f in ("value", "n_gpus", "ranks")} for k in lines}))
    for key in ("dev0", "nodev"):
        two = lines[key]
        assert two["n_gpus"] == 2 and two["ranks"]["world"] == 2 and two["ranks"]["launcher"] == "bench.py"
        assert two["ranks"]["backend"] == "gloo" and len(two["ranks"]["hip_runtime"]) == 1
        assert two["detail"]["accepted_reads"] == one["detail"]["accepted_reads"] > 80_000
        assert two["config"]["reads_per_gpu"] == 50_000
        assert two["ranks"]["host_threads_per_rank"] >= 2
    assert lines["nodev"]["ranks"]["launcher_visible_gpus"] >= 1 and lines["nodev"]["ranks"]["device"] == 0


def test_device_count_without_hip():
    """The rank launcher counts GPUs before it starts its children, so it must
    not start the HIP runtime (a parent holding a GPU context must not fork
    and exec them): imsame_amd.dist.visible_gpus() in a fresh process leaves
    no libamdhip64 mapped and agrees with torch.cuda.device_count(), also
    under HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES."""
    import json
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    count = ("import json, sys; sys.path.insert(0, %r); from imsame_amd.dist import visible_gpus; n = visible_gpus(); "
             "maps = open('/proc/self/maps').read(); print(json.dumps({'n': n, 'hip': 'libamdhip64' in maps, "
             "'torch': 'torch' in sys.modules}))" % repo)
    ref = "import torch; print(torch.cuda.device_count())"
    base = {k: v for k, v in os.environ.items() if k not in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                                             "CUDA_VISIBLE_DEVICES")}
    for extra in ({}, {"HIP_VISIBLE_DEVICES": "0"}, {"ROCR_VISIBLE_DEVICES": "0"}):
        env = dict(base, **extra)
        p = subprocess.run([sys.executable, "-c", count], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           timeout=120)
        assert p.returncode == 0, p.stderr.decode(errors="replace")
        got = json.loads(p.stdout.decode().strip().splitlines()[-1])
        assert not got["hip"] and not got["torch"], got
        t = subprocess.run([sys.executable, "-c", ref], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           timeout=300)
        assert t.returncode == 0, t.stderr.decode(errors="replace")
        print(extra, got, "torch:", t.stdout.decode().strip())
        assert got["n"] == int(t.stdout.decode().strip().splitlines()[-1]) >= 1, (extra, got)


def test_rccl_world1_next_to_library():
    """A world-size-1 RCCL process group with GPU-tensor all-reduces and the
    database-shard merge (imsame_amd.dist) in the same process as the
    library's streams: one HIP runtime mapped, the merge equals the rows,
    and an alignment after the collectives gives the same rows again."""
    import json
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-u", "-m", "tests.rccl_run"], cwd=repo, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:].decode(errors="replace")
    d = json.loads(p.stdout.decode().strip().splitlines()[-1])
    print(d)
    assert d["backend"] == "nccl" and len(d["hip_runtime"]) == 1, d
    assert d["merge_equal"] and d["rerun_equal"], d
    assert d["all_reduce"] == [d["accepted"], d["reads"]] and d["all_reduce_max"] == [1.5], d
    # the bench's own one-rank RCCL form (--dist): its line names the backend
    p = subprocess.run([sys.executable, "-u", "bench.py", "--gpus", "1", "--dist", "--steps", "1", "--warmup", "0",
                        "--cpu-sample", "0", "--e2e", "off", "--reads", "50000"], cwd=repo, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:].decode(errors="replace")
    line = json.loads([x for x in p.stdout.decode().splitlines() if x.startswith("{")][-1])
    print(line["ranks"])
    assert line["ranks"]["backend"] == "rccl" and line["ranks"]["world"] == 1
    assert len(line["ranks"]["hip_runtime"]) == 1 and line["detail"]["accepted_reads"] > 40_000


def test_c3_shard_of_10m_query(dev, oracle_memo):
    """BASELINE configs[2] as an 8-GPU rank holds it: reads [0, 1.25M) of a
    10M-read query, uploaded alone with imsame_dev_set_query_range, aligned
    with the chunk heads of -n_threads 16 over the WHOLE 10M query (rpt =
    625,000: a head inside the shard, none at its end) -- not those of a
    1.25M-read query of its own.  Oracle parity on three windows of the
    shard: its start, the chunk head at read 625,000, its end.  (50 Mbp
    database: the semantics under test is the cut; the reads past the shard
    are filler the device never receives.)"""
    ref, rst = synth.make_reference_arr(50_000_000, 2_000, seed=42)
    n_all, n_sh = 10_000_000, 1_250_000
    q_sh, qs_sh = synth.make_reads_arr(ref, n_sh, 150, seed=44)
    assert len(q_sh) == 150 * n_sh
    q = np.empty(150 * n_all, dtype=np.uint8)
    q[:len(q_sh)] = q_sh
    q[len(q_sh):] = np.frombuffer(b"ACGT", dtype=np.uint8)[np.arange(len(q) - len(q_sh)) % 4]
    qs = np.arange(n_all, dtype=np.uint64) * np.uint64(150)
    dev.index(ref, rst)
    dev.set_query(q, qs, 0, n_sh)
    res, _, _ = dev.align(0, n_sh, n_threads=16)
    assert (res["status"] == 1).mean() > 0.85
    head = n_all // 16
    wins = [(0, 1_500), (head - 750, head + 750), (n_sh - 1_500, n_sh)]
    rc, exp, _ = oracle_memo.align_windows(ref, rst, q, qs, wins, None, 16)
    assert rc == 0
    for (a, b), e in zip(wins, exp):
        assert not _cmp(res[a:b], e), ((a, b), _cmp(res[a:b], e))
    # the same reads as a 1.25M-read query of their own have other chunk heads
    # (rpt 78,125): read 78,125 starts a chunk there, not in the 10M query
    assert n_sh // 16 != head


def test_k19_form_equals_k10_and_oracle(dev, oracle, monkeypatch):
    """The packed kernel's 19-column form (reads of one length, 150: 8 lanes
    per pair, every lane of the wave busy) against the 10-column form on the
    same C2-shaped call -- identical rows and paths -- and the oracle; the
    default runs it (stats.launch_k19), IMSAME_NW_K19=0 does not."""
    ref, rst = synth.make_reference_arr(4_000_000, 2_000, seed=71)
    q, qs = synth.make_reads_arr(ref, 40_000, 150, seed=72, ins=0.002, dele=0.002)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    r19, p19, s19 = dev.align(n_threads=16, want_paths=True)
    monkeypatch.setenv("IMSAME_NW_K19", "0")
    r10, p10, s10 = dev.align(n_threads=16, want_paths=True)
    monkeypatch.delenv("IMSAME_NW_K19")
    assert s19.launch_k19 != 0 and s10.launch_k19 == 0, (hex(s19.launch_k19), hex(s10.launch_k19))
    assert not _cmp(r19, r10), _cmp(r19, r10)
    acc = np.flatnonzero(r19["status"] == 1)
    assert len(acc) > 30_000
    for k in acc[::11]:
        a, b = r19[k], r10[k]
        assert p19[a["path_off"]:a["path_off"] + a["path_len"]].tolist() == \
            p10[b["path_off"]:b["path_off"] + b["path_len"]].tolist(), k
    wins = _windows(len(qs))
    rc, exp, _ = oracle.align_windows(ref, rst, q, qs, wins, None, 16)
    assert rc == 0
    for (a, b), e in zip(wins, exp):
        assert not _cmp(r19[a:b], e), ((a, b), _cmp(r19[a:b], e))


def test_non_acgt_bytes_refused(dev):
    """include/imsame_dev.h: the database and the reads hold only 'A', 'C',
    'G', 'T' -- what IMSAME's loaders keep (IMSAME.c:216-221, :340-345) and
    what the 2-bit codes can tell apart.  An 'N' in the database fails the
    index build, a lowercase base in a read fails the call (the check runs in
    the query's packing kernel; the upload's zero padding is not checked),
    both with IMSAME_E_ARG, and the same inputs with ACGT only align."""
    from imsame_amd import ImsameError
    ref, rst = synth.make_reference_arr(400_000, 2_000, seed=5)
    q, qs = synth.make_reads_arr(ref, 3_000, 150, seed=6)
    bad = ref.copy()
    bad[123_457] = ord("N")
    with pytest.raises(ImsameError) as e:
        dev.index(bad, rst)
    assert e.value.code == abi.IMSAME_E_ARG
    dev.index(ref, rst)
    qb = q.copy()
    qb[int(qs[1_777]) + 5] = ord("a")
    dev.set_query(qb, qs)
    with pytest.raises(ImsameError) as e:
        dev.align(n_threads=16)
    assert e.value.code == abi.IMSAME_E_ARG
    dev.set_query(q, qs)
    res, _, st = dev.align(n_threads=16)
    assert (res["status"] == 1).sum() > 2_000


@pytest.mark.timeout(600)
@pytest.mark.parametrize("shape", ["shard", "c2_lane"])
def test_independent_pipelines_equal_joined_rounds(dev, oracle, shape, monkeypatch):
    """imsame_dev.hip:align_one's independent pipelines: after round 1 the
    reads with round-1 candidates (A, the lane's stream) and round 1b's reads
    (B, stream_b, a host thread of its own) run their later rounds apart, each
    in its own part of the candidate lists.  Every per-read field, every
    accepted path's text and the NW count equal the joined rounds'
    (IMSAME_PIPES=0), with round 1's launch cut into its unpredicted and
    predicted candidates (default) or not (IMSAME_CUT_WEAK=0); the default run
    equals the oracle on three windows; a third of the reads are random (many
    later rounds on both pipelines), and IMSAME_SPEC=2 / IMSAME_SPEC_WEAK=8
    squeeze the pipelines' list parts."""
    n = 125_000 if shape == "shard" else 400_000
    ref, rst = synth.make_reference_arr(8_000_000, 2_000, seed=91)
    q, qs = synth.make_reads_arr(ref, n, 150, seed=92, frac_true=0.67, ins=0.002, dele=0.002)
    dev.index(ref, rst)
    dev.set_query(q, qs)
    monkeypatch.setenv("IMSAME_PIPES", "0")
    base, pb, sb = dev.align(n_threads=16, want_paths=True)
    monkeypatch.setenv("IMSAME_PIPES", "1")           # (by default only lanes of >= 200k reads)
    monkeypatch.setenv("IMSAME_DEBUG_ROUNDS", "1")
    res = None
    for env in [{}, {"IMSAME_CUT_WEAK": "0"}, {"IMSAME_SPEC": "2", "IMSAME_SPEC_WEAK": "8"}]:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        r, pp, st = dev.align(n_threads=16, want_paths=True)
        for k in env:
            monkeypatch.delenv(k)
        assert not _cmp(r, base), (env, _cmp(r, base))
        if not env:
            assert st.n_nw == sb.n_nw, (st.n_nw, sb.n_nw)
            res = r
        for k in np.flatnonzero(base["status"] == 1)[::173]:
            s_ = int(base[k]["db_seq"])
            X = ref[int(rst[s_]):int(rst[s_]) + 2_000].tobytes()
            Y = q[int(qs[k]):int(qs[k]) + int(base[k]["ylen"])].tobytes()
            t1, _ = render(X, Y, r[k], pp[r[k]["path_off"]:r[k]["path_off"] + r[k]["path_len"]])
            t0, _ = render(X, Y, base[k], pb[base[k]["path_off"]:base[k]["path_off"] + base[k]["path_len"]])
            assert t1 == t0, (env, k)
    wins = _windows(len(qs))
    rc, exp, _ = oracle.align_windows(ref, rst, q, qs, wins, None, 16)
    assert rc == 0
    for (a, b), e in zip(wins, exp):
        assert not _cmp(res[a:b], e), ((a, b), _cmp(res[a:b], e))
