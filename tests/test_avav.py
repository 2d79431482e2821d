"""All-vs-all metagenome path (the reference's
bin/all_vs_all_metagenomes_IMSAME.sh) and the multi-threaded FASTA parse
(8(f) row 2).

CPU suite: the oracle replaying the script is pinned to the golden run of the
compiled reference (tests/golden/avav, make_avav_golden.py); the driver's run
plan (naming, order, skip-if-exists) against a restatement of the script's
loop; the parallel parse against the serial one.
GPU suite: imsame_all_vs_all (one job, shards over device contexts, on-device
revComp) against the same golden run, byte for byte for THR = 1.
"""
import ctypes as C
import gzip
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from tests import golden_io as G

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AVAV = os.path.join(REPO, "imsame_amd", "bin", "imsame_all_vs_all")
GOLD = os.path.join(G.GOLDEN, "avav")


def _meta():
    return json.load(open(os.path.join(GOLD, "expected.json")))


def _t1(tag):
    with gzip.open(os.path.join(GOLD, "T1", tag + ".align.gz"), "rb") as f:
        return f.read()


def _check_run(exp, thr, blob):
    if thr == 1:
        assert blob == _t1(exp["tag"]), exp["tag"]
    else:
        heads, bodies = G.record_multisets(blob)
        assert heads == exp["headers"], exp["tag"]
        assert bodies == exp["body_sha1s"], exp["tag"]


def _split_runs(stdout):
    """[INFO] summary lines per run, in run order (each run prints one
    'reads (...) from the query' line and one Jaccard line)."""
    info = G.info_lines(stdout)
    return [info[k:k + 2] for k in range(0, len(info), 2)]


def script_names(base, ext):
    """awk -F ".$EXT" '{print $1}' (all_vs_all_metagenomes_IMSAME.sh:21)."""
    for i in range(len(base)):
        if base[i + 1:i + 1 + len(ext)] == ext and i + 1 + len(ext) <= len(base):
            return base[:i]
    return base


def script_plan(mdir, ext, odir):
    """The script's loop (:28-56) as a list of (query, db, rev, out)."""
    names = [script_names(f, ext) for f in sorted(os.listdir(mdir))
             if f.endswith("." + ext) and not f.startswith(".")]
    plan = []
    for i in range(len(names)):
        for j in range(i + 1, len(names)):
            for rev in (0, 1):
                out = f"{odir}/{names[i]}-{names[j]}{'.r' if rev else ''}.align"
                plan.append(("SKIP", out) if os.path.isfile(out) else
                            ("RUN", f"{mdir}/{names[i]}.{ext}", f"{mdir}/{names[j]}.{ext}", rev, out))
    return plan


def parse_dry_run(stdout):
    plan = []
    for line in stdout.decode().splitlines():
        f = line.split()
        if f[0] == "SKIP":
            plan.append(("SKIP", f[1]))
        elif f[0] == "RUN":
            rev = int("(reverse" in line)
            plan.append(("RUN", f[2], f[4], rev, f[-1]))
    return plan


# ---------------------------------------------------------------- CPU suite
@pytest.mark.parametrize("thr", [1, 3])
def test_oracle_replay_matches_reference_golden(oracle, tmp_path, thr):
    meta = _meta()
    exp_runs = meta["threads"][str(thr)]
    mdir = os.path.join(GOLD, "in")
    k = 0
    for i, X in enumerate(["mgA", "mgB", "mgC"]):
        for Y in ["mgA", "mgB", "mgC"][i + 1:]:
            for rev in (0, 1):
                exp = exp_runs[k]
                k += 1
                db = os.path.join(mdir, f"{Y}.fa")
                if rev:
                    db = str(tmp_path / f"{Y}.r.fa")
                    open(db, "wb").write(oracle.revcomp(open(os.path.join(mdir, f"{Y}.fa"), "rb").read()))
                outp = str(tmp_path / (exp["tag"] + ".align"))
                p = oracle.run_cli(["-query", os.path.join(mdir, f"{X}.fa"), "-db", db, "-n_threads", str(thr),
                                    "-coverage", meta["cov"], "-identity", meta["sim"], "-out", outp])
                assert p.returncode == exp["rc"]
                assert G.info_lines(p.stdout) == exp["info"]
                _check_run(exp, thr, open(outp, "rb").read())
    assert k == len(exp_runs)


def test_driver_usage_error():
    p = subprocess.run([AVAV, "a", "b"], stdout=subprocess.PIPE, timeout=60)
    assert p.returncode == 255
    assert p.stdout.startswith(b"***ERROR*** Use: ")


def test_driver_plan_matches_script_loop(tmp_path):
    mdir, odir = tmp_path / "m", tmp_path / "o"
    mdir.mkdir()
    odir.mkdir()
    for n in ["s2.fasta", "s1.fasta", "a_fasta.fasta", "s3.r.fasta", ".hidden.fasta", "x.fa", "B.fasta"]:
        (mdir / n).write_bytes(b">r\nACGT\n")
    (odir / "s1-s2.align").write_bytes(b"")          # resume: this run is skipped
    (odir / "B-s3.r.r.align").write_bytes(b"")
    p = subprocess.run([AVAV, str(mdir), "0.5", "0.5", "4", "fasta", str(odir), "-dry_run"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=60)
    assert p.returncode == 0, p.stderr
    got = parse_dry_run(p.stdout)
    assert got == script_plan(str(mdir), "fasta", str(odir))
    assert ("SKIP", f"{odir}/s1-s2.align") in got and ("SKIP", f"{odir}/B-s3.r.r.align") in got


def _host_lib():
    import imsame_amd
    H = imsame_amd.host_lib()
    H.host_parse_fasta.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_void_p]
    H.host_parse_fasta_mt.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_uint64, C.c_void_p]
    H.host_free_seqs.argtypes = [C.c_void_p]
    return H


class _Seqs(C.Structure):
    _fields_ = [("seq", C.c_void_p), ("start", C.c_void_p), ("n", C.c_uint64), ("len", C.c_uint64),
                ("brk", C.c_void_p)]


def _parse(H, data, want_brk, threads=None, piece=0):
    src = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    s = _Seqs()
    if threads is None:
        rc = H.host_parse_fasta(src.ctypes.data, len(data), want_brk, C.byref(s))
    else:
        rc = H.host_parse_fasta_mt(src.ctypes.data, len(data), want_brk, threads, piece, C.byref(s))
    assert rc == 0
    seq = C.string_at(s.seq, s.len) if s.len else b""
    st = np.ctypeslib.as_array((C.c_uint64 * (s.n + 1)).from_address(s.start)).copy()
    brk = C.string_at(s.brk, (s.len + 7) // 8) if want_brk and s.len else b""
    H.host_free_seqs(C.byref(s))
    return seq, st, brk


def test_parallel_parse_matches_serial():
    H = _host_lib()
    rng = np.random.default_rng(9)
    alphabet = np.frombuffer(b"ACGTacgtNn-*\r\n\n\n\n>>", np.uint8)
    blobs = [b"", b">", b">x", b"AC\n>x\nAC\n>", b">a\nAC\r\nGT\n>b>c\nTT\n", b"junk\n>a\nAC\n>b\n>\n>c\nGG\n>",
             open(os.path.join(GOLD, "in", "mgC.fa"), "rb").read()]
    for _ in range(30):
        blobs.append(alphabet[rng.integers(0, len(alphabet), int(rng.integers(1, 3000)))].tobytes())
        body = b"".join(b">h%d x>y\n" % k + alphabet[rng.integers(0, 12, int(rng.integers(0, 200)))].tobytes()
                        + b"\n" for k in range(int(rng.integers(1, 40))))
        blobs.append(body)
    for data in blobs:
        for wb in (0, 1):
            ref = _parse(H, data, wb)
            for th, piece in [(2, 1), (3, 7), (8, 64), (16, 1), (5, 0)]:
                got = _parse(H, data, wb, th, piece)
                assert got[0] == ref[0] and np.array_equal(got[1], ref[1]) and got[2] == ref[2], (data[:60], th)


# ---------------------------------------------------------------- GPU suite
@pytest.mark.gpu
@pytest.mark.parametrize("thr,devices", [(1, "1"), (1, "0,0"), (3, "0,0,0")], ids=["T1-1ctx", "T1-2ctx", "T3-3ctx"])
def test_driver_matches_reference_golden(tmp_path, thr, devices):
    meta = _meta()
    mdir, odir = tmp_path / "m", tmp_path / "o"
    shutil.copytree(os.path.join(GOLD, "in"), mdir)
    odir.mkdir()
    p = subprocess.run([AVAV, str(mdir), meta["cov"], meta["sim"], str(thr), "fa", str(odir), "-devices", devices],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    runs = meta["threads"][str(thr)]
    assert _split_runs(p.stdout) == [r["info"] for r in runs]
    for r in runs:
        _check_run(r, thr, (odir / (r["tag"] + ".align")).read_bytes())
    assert sorted(os.listdir(mdir)) == ["mgA.fa", "mgB.fa", "mgC.fa"]      # nothing written there


@pytest.mark.gpu
def test_driver_resumes_skipping_existing_outputs(tmp_path):
    meta = _meta()
    mdir, odir = tmp_path / "m", tmp_path / "o"
    shutil.copytree(os.path.join(GOLD, "in"), mdir)
    odir.mkdir()
    (odir / "mgA-mgC.r.align").write_bytes(b"keep")
    p = subprocess.run([AVAV, str(mdir), meta["cov"], meta["sim"], "1", "fa", str(odir)],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert (odir / "mgA-mgC.r.align").read_bytes() == b"keep"
    runs = [r for r in meta["threads"]["1"] if r["tag"] != "mgA-mgC.r"]
    assert _split_runs(p.stdout) == [r["info"] for r in runs]
    for r in runs:
        _check_run(r, 1, (odir / (r["tag"] + ".align")).read_bytes())
