"""CPU tests of the product's host side and of the kernel SOURCE via the
wave emulator (tests/emu): no GPU needed."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import imsame_amd
from imsame_amd import abi, fasta
from imsame_amd import PARITY_FIELDS
from tests import golden_io as G
from tests import synth
from tests.emu_bind import Emu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "imsame_dev.h")
LIBDEV = os.path.join(REPO, "imsame_amd", "lib", "libimsame_dev.so")


@pytest.fixture(scope="module")
def emu():
    return Emu.load()


def _declared_symbols():
    import re
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char \*)\s*\*?\s*(imsame_\w+)\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIBDEV):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "imsame_amd", "csrc")], check=True)
    lib = C.CDLL(LIBDEV)
    syms = _declared_symbols()
    assert len(syms) >= 9, syms
    for s in syms:
        assert hasattr(lib, s), s


def test_abi_struct_layout():
    assert C.sizeof(abi.ReadResult) == 64
    assert abi.ReadResult.path_len.offset == 60
    assert C.sizeof(abi.Params) == 80
    assert abi.Params.igap.offset == 48


def test_open_without_gpu_fails_loudly():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    import imsame_amd
    with pytest.raises(imsame_amd.ImsameError):
        imsame_amd.Device(0)


def test_fasta_loader_matches_oracle_loader(oracle):
    files = []
    for c in G.e2e_cases():
        d = G.e2e_case(c)
        files += [d["db"], d["query"]]
    rcd = os.path.join(G.GOLDEN, "revcomp")
    files += [os.path.join(rcd, f) for f in sorted(os.listdir(rcd))]
    blobs = [open(f, "rb").read() for f in files] + [
        b"", b">", b">x", b">x\n", b"AC>x\nAC\n>", b">a\nAC\r\nGT\n>b>c\nTT\n",
        b">a\nACGTNACGT\n>b\n\n>c\nacgtx-ACGT\n>"]
    for data in blobs:
        n = len(data)
        src = np.frombuffer(data, np.uint8)
        seq = np.zeros(n + 1, np.uint8)
        st = np.zeros(n + 2, np.uint64)
        bk = np.zeros(n // 8 + 2, np.uint8)
        L, N = C.c_uint64(), C.c_uint64()
        oracle.lib.or_parse(C.c_void_p(src.ctypes.data), C.c_uint64(n), C.c_int(1), C.c_void_p(seq.ctypes.data),
                            C.byref(L), C.c_void_p(st.ctypes.data), C.byref(N), C.c_void_p(bk.ctypes.data))
        s2, st2, b2 = fasta.parse(data, True)
        nb = (L.value + 7) // 8
        assert seq[:L.value].tobytes() == s2.tobytes()
        assert np.array_equal(st[:N.value], st2)
        assert bk[:nb].tobytes() == b2[:nb].tobytes()


@pytest.mark.parametrize("flags", [0, imsame_amd.FLAG_NW32], ids=["auto", "nw32"])
def test_emulated_nw_kernel_matches_reference_golden(emu, oracle, flags):
    """The NW kernel source, run lane by lane, against the reference's NW.
    auto: short reads take the packed-pair int16 kernel (nw16_kernel.hip)
    wherever it fits; nw32: the int32 kernel (nw_kernel.hip) everywhere."""
    rows = [r for r in G.nw_pairs() if len(r["X"]) * len(r["Y"]) <= 80_000]
    assert len(rows) > 200
    groups = {}
    for r in rows:       # short reads (one strip) apart, as imsame_dev_align launches them
        groups.setdefault((r["igap"], r["egap"], len(r["Y"]) <= 160), []).append(r)
    for (ig, eg, _), rs in groups.items():
        p = oracle.params(igap=ig, egap=eg, flags=flags)
        rc, res, _, flags = emu.nw_pairs([r["X"].encode() for r in rs], [r["Y"].encode() for r in rs], p)
        assert rc == 0 and flags == 0
        for k, r in enumerate(rs):
            for f in ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y"):
                assert int(res[k][f]) == r[f], (f, ig, eg, len(r["X"]), len(r["Y"]))


@pytest.mark.parametrize("cols", ["10", "5"])
def test_emulated_packed_nw_mixed_shapes(emu, oracle, cols, monkeypatch):
    """nw16_kernel.hip (emulated) on launches mixing record lengths, read
    lengths (unequal halves of a pair, idle groups) and gap parameters, with
    10 and 5 columns per lane (imsame_dev.hip:nw16_k)."""
    monkeypatch.setenv("IMSAME_NW_K", cols)
    rng = np.random.default_rng(77)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    for ig, eg, mult5 in [(-5, -2, False), (0, 0, False), (-40, -2, False), (-5, -2, True), (-3, -1, True)]:
        X, Y = [], []
        for k in range(11):
            xl = int(rng.choice([12, 13, 40, 150, 333, int(rng.integers(12, 600))]))
            if mult5:       # every read length a multiple of NW16_K: the static-last-column variant
                yl = int(rng.choice([20, 100, 150, 160, 10 * int(rng.integers(2, 17))]))
            else:
                yl = int(rng.choice([12, 31, 100, 149, 150, 160, int(rng.integers(12, 161))]))
            x = acgt[rng.integers(0, 4, xl)]
            if rng.random() < 0.7:
                o = int(rng.integers(0, max(1, xl - yl)))
                y = x[o:o + yl].copy()
                if len(y) < yl:
                    y = np.concatenate([y, acgt[rng.integers(0, 4, yl - len(y))]])
                mut = rng.random(yl) < 0.05
                y[mut] = acgt[rng.integers(0, 4, int(mut.sum()))]
            else:
                y = acgt[rng.integers(0, 4, yl)]
            X.append(x.tobytes()); Y.append(y.tobytes())
        p = oracle.params(igap=ig, egap=eg)
        rc, res, _, flags = emu.nw_pairs(X, Y, p)
        assert rc == 0 and flags == 0
        for k in range(len(X)):
            o = oracle.nw(X[k], Y[k], igap=ig, egap=eg, text=False)
            for f in ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y"):
                assert int(res[k][f]) == int(o[f]), (f, k, ig, eg, len(X[k]), len(Y[k]))


@pytest.mark.parametrize("band,cols", [("200", "10"), ("40", "10"), ("0", "10"), ("200", "5"), ("0", "5"),
                                       ("200", "3"), ("40", "3"), ("0", "3")])
def test_emulated_two_pass_band(emu, oracle, band, cols, monkeypatch):
    """nw16_kernel.hip's two passes (emulated): the score-only sweep with
    checkpoints, then the traceback band restored per half from its own
    checkpoint.  Records long enough that the band starts past row 1; small
    bands make paths leave it, so the waves redo the second sweep from row 1.
    Every field and every path equals the one-pass kernel and the oracle."""
    rng = np.random.default_rng(int(band) + 5)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    X, Y = [], []
    for k in range(9):
        xl = int(rng.integers(250, 700))
        # (the 3-column form takes reads of <= 150 bases: NW16_K3_YMAX)
        yl = int(rng.choice([150, 149, 60, int(rng.integers(20, 151 if cols == "3" else 161))]))
        x = acgt[rng.integers(0, 4, xl)]
        if k % 3 != 2:              # true hits at varied depths (best cells spread over the rows)
            o = int(rng.integers(0, xl - yl))
            y = x[o:o + yl].copy()
            mut = rng.random(yl) < 0.04
            y[mut] = acgt[rng.integers(0, 4, int(mut.sum()))]
            if rng.random() < 0.5:  # an indel run: up / left jumps on the path
                c = int(rng.integers(10, yl - 10))
                y = np.concatenate([y[:c], acgt[rng.integers(0, 4, 3)], y[c:]])[:yl]
        else:
            y = acgt[rng.integers(0, 4, yl)]
        X.append(x.tobytes()); Y.append(y.tobytes())
    monkeypatch.setenv("IMSAME_NW_BAND", band)
    monkeypatch.setenv("IMSAME_NW_K", cols)
    redo = emu.lib.emu_redo_count
    redo.restype = C.c_uint32
    redo()
    p2 = oracle.params(want_paths=1)
    rc, res2, paths2, fl = emu.nw_pairs(X, Y, p2, paths_cap=4096)
    assert rc == 0 and fl == 0
    n_redo = redo()
    if cols == "3":                 # the 3-column latency form ran (mixed lengths: no LAST)
        k3 = emu.lib.emu_k3_count
        k3.restype = C.c_uint32
        assert k3() > 0
    p1 = oracle.params(want_paths=1, flags=imsame_amd.FLAG_NW16_ONEPASS)
    rc, res1, paths1, fl = emu.nw_pairs(X, Y, p1, paths_cap=4096)
    assert rc == 0 and fl == 0 and redo() == 0
    for k in range(len(X)):
        o = oracle.nw(X[k], Y[k], text=False)
        for f in ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y"):
            assert int(res2[k][f]) == int(o[f]) == int(res1[k][f]), (f, k, band, len(X[k]), len(Y[k]))
        if res2[k]["status"] == 1:
            a, b = res2[k], res1[k]
            assert paths2[a["path_off"]:a["path_off"] + a["path_len"]].tolist() == \
                paths1[b["path_off"]:b["path_off"] + b["path_len"]].tolist()
    if band == "0":
        assert n_redo > 0           # a zero band cannot hold a path: the redo path ran
    if band == "200":
        assert n_redo == 0


@pytest.mark.parametrize("band", ["200", "40", "0"])
def test_emulated_k19_form(emu, oracle, band, monkeypatch):
    """nw16_kernel.hip's 19-column form (emulated): launches whose reads all
    have 150 bases run 8 lanes per pair (two padding columns ahead of column
    0 in lane 0, the last column in slot 18), 8 groups per wave, 6 traceback
    dwords per lane per step.  Two passes with bands that hold the path, that
    do not (redo) and none, and one pass: every field equals the oracle and
    every path the 10-column form's; 19 pairs leave idle groups in the last
    wave."""
    rng = np.random.default_rng(int(band) + 19)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    X, Y = [], []
    for k in range(19):
        xl = int(rng.integers(150, 700))
        x = acgt[rng.integers(0, 4, xl)]
        if k % 3 != 2:
            o = int(rng.integers(0, max(1, xl - 150)))
            y = x[o:o + 150].copy()
            if len(y) < 150:
                y = np.concatenate([y, acgt[rng.integers(0, 4, 150 - len(y))]])
            mut = rng.random(150) < 0.04
            y[mut] = acgt[rng.integers(0, 4, int(mut.sum()))]
            if rng.random() < 0.5:                  # an indel run: up / left jumps
                c = int(rng.integers(10, 140))
                y = np.concatenate([y[:c], acgt[rng.integers(0, 4, 3)], y[c:]])[:150]
        else:
            y = acgt[rng.integers(0, 4, 150)]
        X.append(x.tobytes()); Y.append(y.tobytes())
    monkeypatch.setenv("IMSAME_NW_BAND", band)
    k19 = emu.lib.emu_k19_count
    k19.restype = C.c_uint32
    k19()
    out = {}
    k3 = emu.lib.emu_k3_count
    k3.restype = C.c_uint32
    k3()
    # (and the 3-column latency form on the same 150-base reads: its LAST form)
    for form, env in (("k19", None), ("k10", "10"), ("k3", "3")):
        if env:
            monkeypatch.setenv("IMSAME_NW_K", env)
        for one in (False, True):
            p = oracle.params(want_paths=1, flags=imsame_amd.FLAG_NW16_ONEPASS if one else 0)
            rc, res, paths, fl = emu.nw_pairs(X, Y, p, paths_cap=8192)
            assert rc == 0 and fl == 0
            out[form, one] = (res, paths)
        assert (k19() > 0) == (form == "k19")
        assert (k3() > 0) == (form == "k3")
    for k in range(len(X)):
        o = oracle.nw(X[k], Y[k], text=False)
        for key, (res, paths) in out.items():
            for f in ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y"):
                assert int(res[k][f]) == int(o[f]), (key, f, k, band)
        if o["length"] and out["k10", True][0][k]["status"] == 1:
            ref = out["k10", True]
            want = ref[1][ref[0][k]["path_off"]:ref[0][k]["path_off"] + ref[0][k]["path_len"]].tolist()
            for key, (res, paths) in out.items():
                assert paths[res[k]["path_off"]:res[k]["path_off"] + res[k]["path_len"]].tolist() == want, (key, k)


@pytest.mark.parametrize("seed_l,weak_rows", [("1", "0"), ("4", "0"), ("1", "1"), ("4", "1")])
def test_emulated_predicted_traceback_window(emu, oracle, seed_l, weak_rows, monkeypatch):
    """nw16_kernel.hip's predicted window (emulated pipeline): the strong seed
    hit's diagonal (seed_one, or seed_group's re-derivation) orders the queue
    (8-row buckets) and the first sweep writes the traceback of each wave's
    predicted rows; halves whose best cell lies there walk it, the others
    (random reads, reads over a record end, a path that leaves the window)
    fall back to the second sweep.  Reads with indels and edits, 10 % random;
    every field equals the oracle and the run without windows
    (IMSAME_NW_WINDOW=0), and both kinds of half occur."""
    from tests import synth
    monkeypatch.setenv("IMSAME_SEED_L", seed_l)
    monkeypatch.setenv("IMSAME_NW_WINDOW", "1")       # (imsame_dev.hip: on by default)
    monkeypatch.setenv("IMSAME_NW_WEAK_ROWS", weak_rows)   # weak hits predict rows too
    win = emu.lib.emu_win_count
    win.restype = C.c_uint32
    ref, rst = synth.make_reference_arr(240_000, 700, seed=61)
    q, qs = synth.make_reads_arr(ref, 110, 150, seed=62, sub=0.02, ins=0.01, dele=0.01)
    rc0, exp, _ = oracle.align(ref, rst, q, qs, oracle.params(), 4)
    assert rc0 == 0
    win()
    rc, got, _, st = emu.align(ref, rst, q, qs, oracle.params(), 4)
    n_win = win()
    assert rc == 0
    for f in PARITY_FIELDS:
        assert np.array_equal(got[f], exp[f]), f
    acc = int((exp["status"] == 1).sum())
    assert n_win > acc // 2 and n_win < st.n_nw, (n_win, acc, st.n_nw)
    monkeypatch.setenv("IMSAME_NW_WINDOW", "0")
    rc, got0, _, _ = emu.align(ref, rst, q, qs, oracle.params(), 4)
    assert rc == 0 and win() == 0
    for f in PARITY_FIELDS:
        assert np.array_equal(got0[f], exp[f]), f


@pytest.mark.parametrize("r1b,seed_l,rows", [("1", "", "0"), ("0", "", "0"), ("1", "64", "0"), ("0", "64", "0"),
                                             ("1", "", "1"), ("1", "64", "1")])
def test_emulated_round1b(emu, oracle, r1b, seed_l, rows, monkeypatch):
    """Round 1b (imsame_dev.hip:align_one): reads that round 1 paused without
    a candidate (random reads against a 20 Mbp database spend the 32-hit
    budget) scan on at once with weak-first speculation, before round 1's
    NW results, on the device's second stream; both NW launches update the
    same per-read state.  Every field equals the oracle with and without it,
    and the 1b scan took reads over.  seed_l 64: whole-wave scan groups,
    up to SPEC_BIG candidates per read in the later rounds."""
    from tests import synth
    monkeypatch.setenv("IMSAME_ROUND1B", r1b)
    monkeypatch.setenv("IMSAME_NW_R1B_ROWS", rows)        # round 1b's launch ordered by predicted rows,
    monkeypatch.setenv("IMSAME_NW_WEAK_ROWS", rows)       # weak hits predicting them too
    if seed_l:          # whole-wave groups, which emit up to SPEC_BIG per read after round 1
        monkeypatch.setenv("IMSAME_SEED_L", seed_l)
        monkeypatch.delenv("IMSAME_SPEC", raising=False)
    cnt = emu.lib.emu_r1b_count
    cnt.restype = C.c_uint32
    cnt()
    ref, rst = synth.make_reference_arr(20_000_000, 2_000, seed=5)
    q, qs = synth.make_reads_arr(ref, 240, 150, seed=6)
    rc0, exp, _ = oracle.align(ref, rst, q, qs, oracle.params(), 4)
    assert rc0 == 0
    rc, got, _, st = emu.align(ref, rst, q, qs, oracle.params(), 4)
    assert rc == 0
    for f in PARITY_FIELDS:
        assert np.array_equal(got[f], exp[f]), f
    taken = cnt()
    assert (taken > 0) == (r1b == "1"), taken


def _long_pairs(seed, n, ymax, xmax):
    """Long reads (161 .. ymax, strip edges 639-641 included) against records,
    70 % drawn from the record with substitutions and indels, 30 % random."""
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    X, Y = [], []
    for k in range(n):
        xl = int(rng.integers(300, xmax))
        yl = int(rng.choice([161, 170, 639, 640, 641, int(rng.integers(161, ymax))]))
        x = acgt[rng.integers(0, 4, xl)]
        if rng.random() < 0.7:
            o0 = int(rng.integers(0, max(1, xl - yl)))
            src, y = x[o0:o0 + yl], []
            for b in src:
                r = rng.random()
                if r < 0.02:
                    continue                                  # deletion
                if r < 0.04:
                    y.append(acgt[rng.integers(0, 4)])        # insertion
                y.append(acgt[rng.integers(0, 4)] if rng.random() < 0.05 else b)
            y = np.array(y[:yl], dtype=np.uint8)
            if len(y) < yl:
                y = np.concatenate([y, acgt[rng.integers(0, 4, yl - len(y))]])
        else:
            y = acgt[rng.integers(0, 4, yl)]
        X.append(x.tobytes()); Y.append(y.tobytes())
    return X, Y


@pytest.mark.parametrize("band", ["default", "70"])
def test_emulated_long_two_pass_nw_vs_oracle(emu, oracle, band, monkeypatch):
    """nwl_kernel.hip (emulated): reads of 161 .. 1300 columns (1-3 strips of
    640) in the score-only pass with seams and checkpoints, then the walk over
    traceback bands recomputed on demand -- every field, and the .align text
    of every path, equal to the oracle's.  A 70-step band makes every walk
    span many bands (diagonal runs, up- and left-searches resumed across
    them)."""
    if band != "default":
        monkeypatch.setenv("IMSAME_NWL_BAND", band)
    redo = emu.lib.emu_redo_count
    redo.restype = C.c_uint32
    redo()
    for seed, (ig, eg) in ((11, (-5, -2)), (12, (0, 0)), (13, (-3, -1))):
        X, Y = _long_pairs(seed, 5, 1300, 1500)
        p = oracle.params(igap=ig, egap=eg, want_paths=1, min_coverage=1e-9, min_identity=1e-9)
        rc, res, paths, fl = emu.nw_pairs(X, Y, p, paths_cap=100_000)
        assert rc == 0 and fl == 0
        for k in range(len(X)):
            o = oracle.nw(X[k], Y[k], igap=ig, egap=eg, text=True)
            for f in ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y"):
                assert int(res[k][f]) == int(o[f]), (f, k, ig, eg, len(X[k]), len(Y[k]))
            assert res[k]["status"] == 1
            txt, ident = imsame_amd.render(X[k], Y[k], res[k],
                                           paths[res[k]["path_off"]:res[k]["path_off"] + res[k]["path_len"]])
            assert txt == o["text"] and ident == o["identities"], k
    extra = redo()                  # bands beyond one per strip
    assert (extra > 20) if band == "70" else True


@pytest.mark.parametrize("mode", ["nwp", "fallback"])
def test_emulated_packed_long_nw(emu, oracle, mode, monkeypatch):
    """nwp_kernel.hip (emulated): two long reads per wave in int16 halves,
    each lane in its own frame -- every field equal to the oracle's with no
    wave leaving the range proof; with a 4-point spread limit (IMSAME_NWP_S)
    every wave falls back to the int32 nwl_cand and the rows are the same."""
    cnt = emu.lib.emu_nwp_count
    cnt.restype = C.c_uint32
    cnt.argtypes = [C.POINTER(C.c_uint32)]
    fb = C.c_uint32(0)
    cnt(C.byref(fb))
    if mode == "fallback":
        monkeypatch.setenv("IMSAME_NWP_S", "4")
    X, Y = _long_pairs(11, 6, 1300, 1500)
    p = oracle.params(igap=-5, egap=-2, want_paths=1, min_coverage=1e-9, min_identity=1e-9)
    rc, res, paths, fl = emu.nw_pairs(X, Y, p, paths_cap=100_000)
    assert rc == 0 and fl == 0
    assert cnt(C.byref(fb)) == 1
    assert (fb.value == 0) if mode == "nwp" else (fb.value == 3), fb.value
    assert _nwp_violations(emu) == 0
    for k in range(len(X)):
        o = oracle.nw(X[k], Y[k], igap=-5, egap=-2, text=True)
        for f in ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y"):
            assert int(res[k][f]) == int(o[f]), (f, k)
        txt, _ = imsame_amd.render(X[k], Y[k], res[k], paths[res[k]["path_off"]:res[k]["path_off"] + res[k]["path_len"]])
        assert txt == o["text"], k


def _nwp_violations(emu):
    f = emu.lib.emu_nwp_range_violations
    f.restype = C.c_uint64
    return f()


@pytest.mark.parametrize("size", ["short", "full"])
def test_emulated_packed_long_nw_adversarial(emu, oracle, size):
    """nwp_kernel's int16 range proof runs at 64-step block starts
    and relies on drift bounds inside a block.  The emulator checks the
    conclusion at EVERY step (nwp_kernel.hip:nwp_chk: each packed add, sign
    difference and biased decrement a live cell uses must not wrap in its
    half) on pairs built to stress the frames (synth.adversarial_long_pairs:
    12.5 kbp identical, tandem and dinucleotide repeats, a 3 kbp deletion,
    homopolymers, random, a read longer than its record): no violation, and
    every field equal to the oracle's.  "full" runs all of them at the largest
    sizes nwp_fits admits (~7 min of emulation: IMSAME_EMU_FULL=1, log in
    profiles/r5_sanitize/); the default suite runs the repeat pairs cut to 3 kbp."""
    X, Y = synth.adversarial_long_pairs()
    if size == "full":
        if not os.environ.get("IMSAME_EMU_FULL"):
            pytest.skip("IMSAME_EMU_FULL=1: all pairs at full size")
    else:
        X, Y = [X[k][:3000] for k in (1, 2, 4)], [Y[k][:2800] for k in (1, 2, 4)]
    assert emu.lib.emu_nwp_chk_selftest() == 4            # the check sees a wrap of each kind
    cnt = emu.lib.emu_nwp_count
    cnt.restype = C.c_uint32
    cnt.argtypes = [C.POINTER(C.c_uint32)]
    fb = C.c_uint32(0)
    cnt(C.byref(fb))
    _nwp_violations(emu)
    p = oracle.params(igap=-5, egap=-2, min_coverage=1e-9, min_identity=1e-9, max_read_size=14_000)
    rc, res, _, fl = emu.nw_pairs(X, Y, p)
    assert rc == 0 and fl == 0
    assert cnt(C.byref(fb)) == 1
    viol = _nwp_violations(emu)
    print(f"pairs {len(X)}, waves fallen back {fb.value}, wraps {viol}")
    assert viol == 0, (viol, fb.value)
    for k in range(len(X)):
        o = oracle.nw(X[k], Y[k], igap=-5, egap=-2)
        for f in ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y"):
            assert int(res[k][f]) == int(o[f]), (f, k, fb.value)


def test_emulated_packed_long_seams_equal_int32(emu, oracle, monkeypatch, tmp_path):
    """The packed long kernel's seams (absolute T, mf score and l0 of every
    strip's right edge, written from per-lane frames) equal the int32
    nwl_kernel's for every row, including the rows of a partial last block
    (a record of 1100 rows: the last block of each strip has 10 steps) --
    and the rows equal the oracle's."""
    rng = np.random.default_rng(1)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    x = acgt[rng.integers(0, 4, 1100)]
    y = np.concatenate([x[100:], acgt[rng.integers(0, 4, 400)]])
    X, Y = [x.tobytes()], [y.tobytes()]
    p = oracle.params(igap=-5, egap=-2, want_paths=1, min_coverage=1e-9, min_identity=1e-9)
    seams = {}
    for k, on in (("nwp", "1"), ("nwl", "0")):
        monkeypatch.setenv("IMSAME_NWP", on)
        monkeypatch.setenv("IMSAME_EMU_DUMP_SEAM", str(tmp_path / k))
        rc, res, _, fl = emu.nw_pairs(X, Y, p, paths_cap=100_000)
        assert rc == 0 and fl == 0
        o = oracle.nw(X[0], Y[0], igap=-5, egap=-2)
        for f in ("score", "bx", "by", "length", "identities"):
            assert int(res[0][f]) == int(o[f]), (k, f)
        seams[k] = np.fromfile(tmp_path / k, dtype=np.int32)
    xl, SP = len(x), len(x) + 1
    for st in range((len(y) + 639) // 640 - 1):
        for pl in range(3):                   # nwp: planes (T, mf, l0) x halves; nwl: (T, mf, l0)
            a = seams["nwp"][st * 6 * SP + 2 * pl * SP:][:SP][1:xl]
            b = seams["nwl"][st * 3 * SP + pl * SP:][:SP][1:xl]
            assert np.array_equal(a, b), (st, pl, np.nonzero(a != b)[0][:8] + 1)


def _strip_mix_pairs():
    """163- and 400-column reads in ONE launch: the launch takes the
    multi-strip kernel (ymax > 320) and the 163-column reads have one strip."""
    rng = np.random.default_rng(3)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    X, Y = [], []
    for k in range(6):
        xl = 359 if k == 0 else int(rng.integers(300, 600))
        yl = 163 if k % 2 == 0 else 400
        x = acgt[rng.integers(0, 4, xl)]
        o0 = int(rng.integers(0, max(1, xl - yl)))
        y = np.concatenate([x[o0:o0 + yl], acgt[rng.integers(0, 4, max(0, yl - (xl - o0)))]])[:yl].copy()
        m = rng.random(yl) < 0.05
        y[m] = acgt[rng.integers(0, 4, int(m.sum()))]
        X.append(x.tobytes()); Y.append(y.tobytes())
    return X, Y


def test_emulated_single_strip_reads_in_multi_strip_launch(emu, oracle):
    """nw_kernel.hip MULTI: a read of one strip has no seam (its lead lane is
    column 0).  The emulator's seam buffer is poisoned like fresh device
    memory, so a read of it shows (round 1 read it: wrong scores there)."""
    X, Y = _strip_mix_pairs()
    rc, res, _, fl = emu.nw_pairs(X, Y, oracle.params())
    assert rc == 0 and fl == 0
    for k in range(len(X)):
        o = oracle.nw(X[k], Y[k], text=False)
        for f in ("score", "bx", "by", "length", "identities", "igaps", "egaps", "head_x", "head_y"):
            assert int(res[k][f]) == int(o[f]), (f, k, len(Y[k]))


def _emu_ungapped(emu, db, dbs, q, qs, pd0, pq0, read, sid):
    f = emu.lib.emu_ungapped
    f.restype = C.c_uint64
    u8, u64 = C.POINTER(C.c_uint8), C.POINTER(C.c_uint64)
    f.argtypes = [u8, C.c_uint64, u64, C.c_uint64, u8, C.c_uint64, u64, C.c_uint64] + [C.c_uint64] * 4
    return f(db.ctypes.data_as(u8), len(db), dbs.ctypes.data_as(u64), len(dbs), q.ctypes.data_as(u8), len(q),
             qs.ctypes.data_as(u64), len(qs), pd0, pq0, read, sid)


def test_emulated_ungapped_matches_reference_golden(emu, oracle):
    """seed_kernel.hip:ungapped_raw (16-byte chunked walk) == the reference's
    byte walk on every golden hit, plus random hits incl. buffer starts."""
    rows, cases = G.ungapped_rows()
    arrs = {c: (G.seqs_arrays(v["db"]), G.seqs_arrays(v["reads"])) for c, v in cases.items()}
    for r in rows:
        (db, dbs), (q, qs) = arrs[r["case"]]
        exp = oracle.ungapped(db, dbs, q, qs, r["pos_db"], r["pos_q"], r["read"], r["dbseq"]).raw
        got = _emu_ungapped(emu, db, dbs, q, qs, r["pos_db"], r["pos_q"], r["read"], r["dbseq"])
        assert got == exp, r
    from tests import synth
    rng = np.random.default_rng(5)
    ref, rst = synth.make_reference_arr(60_000, 700, seed=9)
    q, qs = synth.make_reads_arr(ref, 300, 120, seed=10)
    n = 0
    for _ in range(3000):
        sid = int(rng.integers(len(rst)))
        rd = int(rng.integers(len(qs)))
        xs, xe = int(rst[sid]), (int(rst[sid + 1]) if sid + 1 < len(rst) else len(ref))
        ys, ye = int(qs[rd]), (int(qs[rd + 1]) if rd + 1 < len(qs) else len(q))
        if xe - xs < 13 or ye - ys < 13:
            continue
        if rng.random() < 0.5:      # true-hit diagonal: the read's own origin, long extensions
            pq0 = int(rng.integers(ys + 12, ye + 1))
            pd0 = int(rng.integers(xs + 12, xe + 1))
        else:                       # buffer starts and record edges
            pq0 = ys + 12 + int(rng.integers(0, 3))
            pd0 = xs + 12 + int(rng.integers(0, 20))
        exp = oracle.ungapped(ref, rst, q, qs, pd0, pq0, rd, sid).raw
        assert _emu_ungapped(emu, ref, rst, q, qs, pd0, pq0, rd, sid) == exp, (pd0, pq0, rd, sid)
        n += 1
    assert n > 2000
    # exact matches far past one 16-byte chunk in both directions
    q2 = ref[1000:1400].copy()
    qs2 = np.array([0], dtype=np.uint64)
    sid = int(np.searchsorted(rst, 1000, side="right") - 1)
    for off in (12, 13, 40, 200, 399, 400):
        exp = oracle.ungapped(ref, rst, q2, qs2, 1000 + off, off, 0, sid).raw
        assert _emu_ungapped(emu, ref, rst, q2, qs2, 1000 + off, off, 0, sid) == exp
    # true diagonals with sparse mismatches (walks of many chunks that stop
    # anywhere in an 8-step table row, or run into a read's or a record's end
    # inside a chunk), every seed position of reads of ragged lengths
    base = 20_000
    src = ref[base:base + 1200].copy()
    for rate in (0.03, 0.12, 0.3):
        q3 = src.copy()
        mm = rng.random(len(q3)) < rate
        q3[mm] = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, int(mm.sum()))]
        cuts = np.sort(rng.choice(np.arange(20, len(q3) - 20), 9, replace=False))
        qs3 = np.concatenate([[0], cuts]).astype(np.uint64)
        for rd in range(len(qs3)):
            ys = int(qs3[rd])
            ye = int(qs3[rd + 1]) if rd + 1 < len(qs3) else len(q3)
            for pq0 in range(ys + 12, ye + 1, 3):
                pd0 = base + pq0
                sid = int(np.searchsorted(rst, pd0 - 12, side="right") - 1)
                if int(rst[sid]) > pd0 - 12 or (sid + 1 < len(rst) and int(rst[sid + 1]) < pd0):
                    continue                # seeds lie inside one record
                exp = oracle.ungapped(ref, rst, q3, qs3, pd0, pq0, rd, sid).raw
                assert _emu_ungapped(emu, ref, rst, q3, qs3, pd0, pq0, rd, sid) == exp, (rate, rd, pq0)
                n += 1
    assert n > 2600


@pytest.mark.parametrize("flags", [0, imsame_amd.FLAG_NW32], ids=["auto", "nw32"])
@pytest.mark.parametrize("name", ["borrowed", "edges", "reads_vs_reads", "toolong"])
def test_emulated_pipeline_matches_oracle(emu, oracle, name, flags, monkeypatch):
    """Seed scan + rounds + NW (kernel source, emulated) vs the oracle.
    (Single-lane scan here; the grouped scan: test_emulated_pipeline_seed_budget.)"""
    monkeypatch.setenv("IMSAME_SEED_L", "1")
    case = G.e2e_case(name)
    db, dbs, brk = fasta.load(case["db"], True)
    q, qs, _ = fasta.load(case["query"])
    runs = [int(t) for t in case["meta"]["runs"]]
    if name == "edges":             # 3 kbp reads x 3 kbp records: minutes per run in the emulator
        runs = [runs[0], runs[-1]]
    for T in runs:
        p = oracle.params()
        rc1, r1, er = oracle.align(db, dbs, q, qs, p, T, brk)
        p.flags = flags
        rc2, r2, _, st = emu.align(db, dbs, q, qs, p, T, db_brk=brk)
        assert rc1 == rc2
        n = er if rc1 else len(r1)
        for f in PARITY_FIELDS:
            assert np.array_equal(r1[f][:n], r2[f][:n]), (name, T, f)
        if rc1:
            assert st.err_read == er


@pytest.mark.parametrize("budget,lanes,spec,weak,rel", [
    ("1", "1", "8", "4", "0"), ("3", "1", "1", "1", "0"), ("0", "4", "8", "8", "0"), ("3", "4", "2", "4", "0"),
    ("1", "16", "8", "2", "0"), ("0", "16", "1", "8", "0"), ("0", "1", "1", "8", "0"), ("1", "64", "8", "4", "0"),
    ("3", "64", "2", "1", "0"), ("1", "1", "8", "4", "1"), ("3", "4", "2", "4", "1"), ("1", "64", "8", "4", "1")])
def test_emulated_pipeline_seed_budget(emu, oracle, budget, lanes, spec, weak, rel, monkeypatch):
    """Reads that pause on the per-round hit budget resume at the same hit,
    the grouped scan (L lanes per read, seed_kernel.hip:seed_group) merges
    its windows in visiting order, and speculative candidates after a
    rejection (up to `spec` per read and round) or from a weak first
    candidate on (up to `weak`, seed_kernel.hip:spec_after_first) keep the
    first accepted one in visiting order: results equal the oracle's for
    every budget (0 = none), group size and speculation width, with the
    index entries in either form (rel: IMSAME_ENT_REL, seed_kernel.hip:ent_pos)."""
    monkeypatch.setenv("IMSAME_ENT_REL", rel)
    monkeypatch.setenv("IMSAME_SEED_BUDGET", budget)
    monkeypatch.setenv("IMSAME_SEED_L", lanes)
    monkeypatch.setenv("IMSAME_SPEC", spec)
    monkeypatch.setenv("IMSAME_SPEC_WEAK", weak)
    r1b = emu.lib.emu_r1b_count
    r1b.restype = C.c_uint32
    r1b()
    rounds = 0
    for name in ("borrowed", "reads_vs_reads", "toolong"):
        case = G.e2e_case(name)
        db, dbs, brk = fasta.load(case["db"], True)
        q, qs, _ = fasta.load(case["query"])
        T = int(list(case["meta"]["runs"])[-1])
        rc1, r1, er = oracle.align(db, dbs, q, qs, oracle.params(), T, brk)
        rc2, r2, _, st = emu.align(db, dbs, q, qs, oracle.params(), T, db_brk=brk)
        assert rc1 == rc2
        n = er if rc1 else len(r1)
        for f in PARITY_FIELDS:
            assert np.array_equal(r1[f][:n], r2[f][:n]), (name, budget, f)
        rounds = max(rounds, st.rounds)
    # a budget pauses reads: they resume in round 2, or in round 1b (the
    # device's policy, round_policy.h, gives small calls round 2's budget x 64)
    assert rounds >= 2 or r1b() > 0 or budget == "0", rounds


@pytest.mark.parametrize("spec,weak", [("1", "1"), ("8", "8")])
def test_emulated_nw_accounting(emu, oracle, spec, weak, monkeypatch):
    """The device's NW work against the reference's (alignmentFunctions.c:
    126-186: one NW per e-value-passing hit until one is accepted): n_nw minus
    the speculative candidates past each read's accepted one
    (imsame_stats.nw_spec_waste, update_one) equals the oracle's count of
    distinct (read, record) NWs, and the oracle without its memo -- the
    reference's own count -- is at least that.  Without speculation nothing
    is wasted."""
    import ctypes
    from tests import synth
    monkeypatch.setenv("IMSAME_SPEC", spec)
    monkeypatch.setenv("IMSAME_SPEC_WEAK", weak)
    oracle.lib.or_last_nw.restype = ctypes.c_uint64
    ref, rst = synth.make_reference_arr(400_000, 2_000, seed=71)
    q, qs = synth.make_reads_arr(ref, 400, 150, seed=72)
    rc2, r2, _, st = emu.align(ref, rst, q, qs, oracle.params(), 4)
    oracle.lib.or_set_memo_rejected(1)
    try:
        rc1, r1, _ = oracle.align(ref, rst, q, qs, oracle.params(), 4)
        distinct = int(oracle.lib.or_last_nw())
    finally:
        oracle.lib.or_set_memo_rejected(0)
    rc0, r0, _ = oracle.align(ref, rst, q, qs, oracle.params(), 4)
    reference = int(oracle.lib.or_last_nw())
    assert rc0 == rc1 == rc2 == 0
    for f in PARITY_FIELDS:
        assert np.array_equal(r1[f], r2[f]) and np.array_equal(r0[f], r1[f]), f
    assert st.n_nw - st.nw_spec_waste == distinct, (st.n_nw, st.nw_spec_waste, distinct)
    assert reference >= distinct > 0
    if spec == weak == "1":
        assert st.nw_spec_waste == 0


def test_thresholds_match_long_double_tests(emu, oracle):
    """Integer tables (csrc/tables.h) == the reference's long double tests."""
    lib = emu.lib
    lib.emu_minraw.restype = C.c_uint64
    lib.emu_minraw.argtypes = [C.c_uint64, C.c_uint64, C.POINTER(abi.Params)]
    lib.emu_minnum.restype = C.c_uint32
    lib.emu_minnum.argtypes = [C.c_uint64, C.c_uint64, C.POINTER(abi.Params), C.c_int]
    oracle.lib.or_epass.restype = C.c_int
    oracle.lib.or_epass.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(abi.Params)]
    for p in (oracle.params(), oracle.params(min_e=1e-10), oracle.params(min_e=1e-30),
              oracle.params(min_e=0.0)):
        for L in (1_000_000, 50_000_000, 500_000_000):
            for y in list(range(0, 40)) + [99, 100, 101, 149, 150, 151, 1000, 2999, 3000]:
                m = lib.emu_minraw(y, L, C.byref(p))
                for raw in list(range(0, 8 * y + 80, 4)) + [m - 1, m, m + 1, 2**63, 2**64 - 1]:
                    if raw < 0 or raw >= 2**64:
                        continue
                    exp = oracle.lib.or_epass(raw, y, L, C.byref(p))
                    assert (m != 2**64 - 1 and raw >= m) == bool(exp), (y, L, raw, m)
    p = oracle.params(min_coverage=0.5, min_identity=0.9)
    for den in range(1, 400):
        mc = lib.emu_minnum(den, 2 * den + 8, C.byref(p), 0)
        mi = lib.emu_minnum(den, den, C.byref(p), 1)
        for num in range(0, 2 * den + 8):
            assert (num >= mc) == (num / den >= 0.5)
            if num <= den:
                assert (num >= mi) == bool(oracle.lib.or_ident_ok(num, den, C.byref(p)))


@pytest.mark.parametrize("rec_bp,expect_nw", [(90, False), (200, True)])
def test_emulated_a_priori_rejection(emu, oracle, rec_bp, expect_nw):
    """seed_kernel.hip:nw_cannot_accept / hit_irrelevant / read_irrelevant --
    with 400 bp reads, acceptance needs >= 0.5 * 0.5 * 400 = 100 identities,
    more than a 90 bp record can give, so every hit is dropped without an
    extension or NW (the oracle runs and rejects each NW); at 200 bp records
    NW runs.  Results equal the oracle's."""
    from tests import synth
    ref, rst = synth.make_reference_arr(12_000, rec_bp, seed=13)
    q, qs = synth.make_reads_arr(ref, 2, 400, seed=14)
    rc1, r1, _ = oracle.align(ref, rst, q, qs, oracle.params(), 3)
    rc2, r2, _, st = emu.align(ref, rst, q, qs, oracle.params(), 3)
    assert rc1 == rc2 == 0
    for f in PARITY_FIELDS:
        assert np.array_equal(r1[f], r2[f]), f
    assert (st.n_nw > 0) == expect_nw


@pytest.mark.parametrize("name", ["empty_not_head", "borrowed", "edges"])
def test_emulated_query_shards_equal_whole_run(emu, oracle, name, monkeypatch):
    """imsame_dev_set_query_range semantics (the emulator uploads ONLY the
    shard's reads and poisons everything else): two shards split at every
    read (empty reads right before a shard, chunk heads outside it, the
    borrowed base across the cut) concatenate to the oracle's whole-query
    run, for every -n_threads of the golden case."""
    monkeypatch.setenv("IMSAME_SEED_L", "1")
    case = G.e2e_case(name)
    db, dbs, brk = fasta.load(case["db"], True)
    q, qs, _ = fasta.load(case["query"])
    n = len(qs)
    cuts = range(1, n) if n <= 12 else sorted({1, n // 2, n - 1})
    for T in [int(list(case["meta"]["runs"])[-1])]:        # the most chunk heads
        rc, exp, er = oracle.align(db, dbs, q, qs, oracle.params(), T, brk)
        if rc:
            continue                      # the size abort: covered by the pipeline tests
        for k in cuts:
            parts = []
            for a, b in ((0, k), (k, n)):
                rc2, r, _, _ = emu.align(db, dbs, q, qs, oracle.params(), T, read_from=a, read_to=b, db_brk=brk)
                assert rc2 == 0
                parts.append(r)
            got = np.concatenate(parts)
            for f in PARITY_FIELDS:
                assert np.array_equal(got[f], exp[f]), (name, T, k, f)


def test_render_of_emulated_paths_matches_reference_text(emu, oracle):
    """host_render (the CLI's .align text, alignmentFunctions.c:210-274, with
    scratch reused across records) from paths the kernel source produces:
    the reference's text bytes (SHA-1 of the golden pairs) and identities."""
    import hashlib
    rows = [r for r in G.nw_pairs() if len(r["X"]) * len(r["Y"]) <= 60_000 and r["igap"] == -5 and r["egap"] == -2]
    rows = [r for r in rows if len(r["Y"]) <= 160][:60]
    assert len(rows) > 20
    p = oracle.params(min_coverage=1e-9, min_identity=1e-9)
    p.want_paths = 1
    X = [r["X"].encode() for r in rows]
    Y = [r["Y"].encode() for r in rows]
    rc, res, paths, flags = emu.nw_pairs(X, Y, p, paths_cap=sum(len(x) + len(y) for x, y in zip(X, Y)) + 16)
    assert rc == 0 and flags == 0
    n = 0
    for k, r in enumerate(rows):
        if res[k]["status"] != 1:
            continue
        pk = paths[res[k]["path_off"]:res[k]["path_off"] + res[k]["path_len"]]
        txt, ident = imsame_amd.render(X[k], Y[k], res[k], pk)
        assert hashlib.sha1(txt).hexdigest() == r["text_sha1"], k
        assert ident == r["identities"]
        n += 1
    assert n > 20
