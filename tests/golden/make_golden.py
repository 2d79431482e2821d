#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ from the REFERENCE itself.

The reference (Bitlab-UMA/IMSAME) ships no tests, fixtures or golden files
(SURVEY.md section 4), so every parity pin is produced here by running the
reference compiled from its own sources (oracle/Makefile `ref` target ->
oracle/_ref/{IMSAME,revComp,ref_driver}) on synthetic inputs.  Only this
container has /root/reference; the fixtures are committed and travel.

    python tests/golden/make_golden.py        # (re)writes the fixtures

Fixtures (data only -- inputs and the reference's outputs):
  nw_pairs.jsonl.gz   unit NW + backtracking + text (alignmentFunctions.c:210-560)
  ungapped.jsonl.gz   alignmentFromQuickHits outputs incl. the long double e-value
  e2e/<case>/         FASTA inputs + the reference's .align and [INFO] summary
                      for -n_threads 1 (file order) and 2/4/7 (record multisets)
  revcomp/<case>.*    revComp input / output pairs
"""
import gzip
import hashlib
import json
import os
import re
import shutil
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref")
sys.path.insert(0, REPO)
from tests.synth import make_reference, make_reads  # noqa: E402
from tests.golden_io import record_multisets  # noqa: E402

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def rand_seq(rng, n):
    return ACGT[rng.integers(0, 4, n)].tobytes().decode()


def mutate(rng, s, sub, ins, dele):
    out = []
    for c in s:
        r = rng.random()
        if r < dele:
            continue
        if r < dele + ins:
            out.append("ACGT"[rng.integers(0, 4)])
        if rng.random() < sub:
            c = "ACGT".replace(c, "")[rng.integers(0, 3)]
        out.append(c)
    return "".join(out)


def build_ref():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)


# ---------------------------------------------------------------- NW ------
def nw_cases(rng):
    cases = []
    # (xlen range, ylen range, kind, count)
    plan = [
        ((12, 40), (11, 40), "rand", 60),
        ((12, 40), (11, 40), "sim95", 60),
        ((40, 400), (20, 160), "rand", 40),
        ((40, 400), (20, 160), "sim70", 40),
        ((40, 400), (20, 160), "sub95", 40),
        ((1500, 2100), (100, 151), "embed", 30),   # C1/C2-like: read inside a record
        ((100, 160), (100, 160), "sim90", 30),     # C4-like: read vs read
        ((12, 20), (60, 200), "rand", 10),         # xlen < ylen
        ((2990, 3000), (140, 160), "embed", 4),
        ((2999, 3000), (2999, 3000), "sim90", 2),   # maximum sizes
        ((200, 400), (400, 800), "sim70", 6),
    ]
    gaps = [(-5, -2), (-5, -2), (-5, -2), (-1, -1), (-10, -3), (-2, -4), (0, 0), (-20, -1)]
    for (xr, yr, kind, cnt) in plan:
        for _ in range(cnt):
            xl = int(rng.integers(xr[0], xr[1] + 1))
            yl = int(rng.integers(yr[0], yr[1] + 1))
            ig, eg = gaps[int(rng.integers(0, len(gaps)))]
            x = rand_seq(rng, xl)
            if kind == "rand":
                y = rand_seq(rng, yl)
            elif kind == "embed":
                off = int(rng.integers(0, max(1, xl - yl)))
                y = mutate(rng, x[off:off + yl], 0.01, 0.005, 0.005)
                if len(y) < 11:
                    y = rand_seq(rng, yl)
            else:
                pct = int(kind[-2:]) / 100.0
                src = x[:yl] if len(x) >= yl else x + rand_seq(rng, yl - len(x))
                if kind.startswith("sub"):
                    y = mutate(rng, src, 1 - pct, 0, 0)
                else:
                    y = mutate(rng, src, (1 - pct) * 0.6, (1 - pct) * 0.2, (1 - pct) * 0.2)
                if len(y) < 11:
                    y = y + rand_seq(rng, 11)
            cases.append((ig, eg, x[:3000], y[:3000]))
    # hand-made corner cases
    cases += [
        (-5, -2, "A" * 12, "A" * 11),
        (-5, -2, "ACGTACGTACGT", "TTTTTTTTTTTT"),
        (-5, -2, "AAAAAAAAAAAAAAAAAAAAAAAA", "AAAAAAAAAAAA"),
        (-5, -2, "ACGT" * 30, "ACGT" * 10),
        (-5, -2, "ACGTTGCA" * 40, "TGCA" * 20),
        (-1, 0, "ACGTACGTAAAACCCCGGGGTTTT" * 4, "AAAACCCCGGGGTTTT" * 3),
        (3, 1, "ACGTACGTAAAACCCCGGGGTTTT" * 4, "AAAACCCCGGGGTTTT" * 3),  # positive gap scores
    ]
    return cases


def gen_nw(rng):
    cases = nw_cases(rng)
    p = subprocess.Popen([os.path.join(REF, "ref_driver")], stdin=subprocess.PIPE, stdout=subprocess.PIPE)
    inp = "".join(f"nw {ig} {eg} {x} {y}\n" for (ig, eg, x, y) in cases).encode()
    out, _ = p.communicate(inp)
    assert p.returncode == 0
    rows = []
    pos = 0
    for (ig, eg, x, y) in cases:
        nl = out.index(b"\n", pos)
        f = out[pos:nl].split()
        score, bx, by, length, ident, igaps, egaps, hx, hy, tl = [int(v) for v in f]
        text = out[nl + 1:nl + 1 + tl]
        pos = nl + 1 + tl + 1
        row = dict(igap=ig, egap=eg, X=x, Y=y, score=score, bx=bx, by=by, length=length,
                   identities=ident, igaps=igaps, egaps=egaps, head_x=hx, head_y=hy,
                   text_len=tl, text_sha1=hashlib.sha1(text).hexdigest())
        if tl <= 4000:
            row["text"] = text.decode()
        rows.append(row)
    with gzip.open(os.path.join(HERE, "nw_pairs.jsonl.gz"), "wt") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
    print(f"nw_pairs: {len(rows)}")


# ---------------------------------------------------------- ungapped ------
def kmer_hits(db_recs, q_reads, max_hits):
    """(pos_db, pos_q, read, dbseq) for 12-mer seeds shared by query and DB
    (pos = last base + 1, as the reference's index, IMSAME.c:247)."""
    idx = {}
    off = 0
    for s, rec in enumerate(db_recs):
        for e in range(11, len(rec)):
            idx.setdefault(rec[e - 11:e + 1], []).append((off + e + 1, s))
        off += len(rec)
    qcat = "".join(q_reads)
    qstart = np.cumsum([0] + [len(r) for r in q_reads])
    hits = []
    for r in range(len(q_reads)):
        for p in range(max(11, qstart[r] - 1 + 11), qstart[r + 1]):
            for (pd, s) in idx.get(qcat[p - 11:p + 1], []):
                hits.append((pd, p + 1, r, s))
    return hits[:max_hits]


def gen_ungapped(rng):
    rows = []
    for case in range(6):
        L = [150, 400, 2000, 60, 900, 3000][case]
        nrec = [5, 4, 3, 20, 6, 2][case]
        recs = [rand_seq(rng, int(rng.integers(L // 2, L + 1))) for _ in range(nrec)]
        cat = "".join(recs)
        reads = []
        for k in range(12):
            rl = int(rng.integers(11, 160))
            if k % 3 == 2:
                reads.append(rand_seq(rng, rl))
            else:
                o = int(rng.integers(0, max(1, len(cat) - rl)))
                reads.append(mutate(rng, cat[o:o + rl], [0.0, 0.02, 0.1][k % 3], 0.0, 0.0) or "ACGTACGTACGT")
        hits = kmer_hits(recs, reads, 400)
        # also seeds in odd places: borrowed-base windows and record edges
        p = subprocess.Popen([os.path.join(REF, "ref_driver")], stdin=subprocess.PIPE, stdout=subprocess.PIPE)
        cmd = f"db {len(recs)} " + " ".join(recs) + "\n" + f"q {len(reads)} " + " ".join(reads) + "\n"
        cmd += "".join(f"ug {pd} {pq} {r} {s}\n" for (pd, pq, r, s) in hits)
        out, _ = p.communicate(cmd.encode())
        assert p.returncode == 0
        lines = out.decode().strip().split("\n") if hits else []
        for (pd, pq, r, s), ln in zip(hits, lines):
            xs, ys, tl, ehex, edec = ln.split()
            rows.append(dict(case=case, pos_db=pd, pos_q=pq, read=r, dbseq=s, x_start=int(xs),
                             y_start=int(ys), t_len=int(tl), e_hex=ehex, e_dec=edec))
        with gzip.open(os.path.join(HERE, f"ungapped_case{case}.json.gz"), "wt") as f:
            json.dump(dict(db=recs, reads=reads), f)
    with gzip.open(os.path.join(HERE, "ungapped.jsonl.gz"), "wt") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
    print(f"ungapped: {len(rows)}")


# --------------------------------------------------------------- e2e ------
INFO_RE = re.compile(rb"^\[INFO\] (\d+ reads .*|The Jaccard-index is: .*)$", re.M)


def run_ref_imsame(q, d, out, T, extra=()):
    cmd = [os.path.join(REF, "IMSAME"), "-query", q, "-db", d, "-out", out, "-n_threads", str(T), *extra]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    return p.returncode, p.stdout


def split_records(blob):
    """.align -> list of (header, body) using the fixed header shape."""
    parts = re.split(rb"(\(\d+, \d+\) : \d+% \d+% \d+\n \$\$\$\$\$\$\$ \n)", blob)
    return parts


def e2e_case(name, db_text, q_text, Ts=(1, 2, 4, 7), extra=()):
    d = os.path.join(HERE, "e2e", name)
    if os.path.isdir(d):
        shutil.rmtree(d)
    os.makedirs(d)
    dbp, qp = os.path.join(d, "db.fa"), os.path.join(d, "query.fa")
    with open(dbp, "wb") as f:
        f.write(db_text)
    with open(qp, "wb") as f:
        f.write(q_text)
    meta = dict(extra=list(extra), runs={})
    for T in Ts:
        outp = os.path.join("/tmp", f"golden_{name}_{T}.align")
        rc, so = run_ref_imsame(qp, dbp, outp, T, extra)
        blob = open(outp, "rb").read() if os.path.exists(outp) else b""
        heads = sorted(h.decode() for h in re.findall(rb"\(\d+, \d+\) : \d+% \d+% \d+\n", blob))
        run = dict(rc=rc, info=[m.decode() for m in INFO_RE.findall(so)],
                   err=[l.decode() for l in so.split(b"\n") if l.startswith(b"ERR")],
                   headers=heads, align_sha1=hashlib.sha1(blob).hexdigest(), align_len=len(blob))
        if T == 1:
            with gzip.open(os.path.join(d, "T1.align.gz"), "wb") as f:
                f.write(blob)
        else:
            # bodies of different threads may interleave: keep the body multiset
            run["body_sha1s"] = record_multisets(blob)[1]
        meta["runs"][str(T)] = run
        os.remove(outp) if os.path.exists(outp) else None
    with open(os.path.join(d, "expected.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"e2e {name}: " + ", ".join(f"T{T}:{len(meta['runs'][str(T)]['headers'])}" for T in Ts))


def fasta(recs, width=80, nl=b"\n", prefix="s"):
    out = []
    for i, r in enumerate(recs):
        out.append(f">{prefix}_{i}".encode() + nl)
        rb_ = r.encode() if isinstance(r, str) else r
        if width:
            for k in range(0, len(rb_), width):
                out.append(rb_[k:k + width] + nl)
        else:
            out.append(rb_ + nl)
    return b"".join(out)


def gen_e2e(rng):
    # 1) canonical small synthetic (C1-like, scaled down): 100 kbp in 2 kbp records, 200 reads
    ref = make_reference(100_000, 2_000, seed=7)
    reads = make_reads(ref, 200, 150, seed=8)
    e2e_case("small_c2like", fasta(ref), fasta(reads, width=0, prefix="read"))
    # 2) 100 bp reads (C1 shape)
    reads = make_reads(ref, 150, 100, seed=9)
    e2e_case("small_c1like", fasta(ref), fasta(reads, width=0, prefix="read"))
    # 3) edge cases: N in DB and query, lowercase, multi-line, empty reads, short reads
    ref = make_reference(20_000, 1_000, seed=11)
    recs = [r for r in ref]
    recs[3] = recs[3][:400] + "NNNNN" + recs[3][400:]
    recs[5] = recs[5].lower()
    recs.insert(7, "")                               # empty DB record
    reads = make_reads(ref, 60, 120, seed=12)
    reads[3] = reads[3][:50] + "N" + reads[3][50:]   # N inside a read
    reads[4] = reads[4].lower()
    reads[10] = ""                                    # empty read (not a chunk head for T in 1,2,4,7)
    reads[11] = reads[11][:12]                       # length 12
    reads[12] = reads[12][:13]
    reads[13] = reads[13][:11]
    reads[-1] = reads[-1][:11]                       # last read of length 11
    e2e_case("edges", fasta(recs, width=60), fasta(reads, width=50, prefix="read"))
    # 4) borrowed-base case: 2 reads; read 1's first k-mer uses read 0's last base
    # (SURVEY Appendix A Q4): record 0 holds b+read1, record 1 holds b'+read1.
    # T=1: read 1's first k-mer borrows b -> only record 0 matches -> (1, 0).
    # T=2: read 1 is a chunk head -> its first k-mer hits both, LIFO -> (1, 1).
    r1 = rand_seq(rng, 90)
    b = "A"
    x0 = rand_seq(rng, 200) + b + r1 + rand_seq(rng, 200)
    x1 = rand_seq(rng, 200) + "C" + r1 + rand_seq(rng, 200)
    r0 = rand_seq(rng, 40) + b
    e2e_case("borrowed", fasta([x0, x1]), fasta([r0, r1], width=0, prefix="read"), Ts=(1, 2))
    # 5) CRLF database (k-mers reset at every '\r')
    ref = make_reference(8_000, 1_000, seed=13)
    reads = make_reads(ref, 30, 100, seed=14)
    e2e_case("crlf_db", fasta(ref, width=60, nl=b"\r\n"), fasta(reads, width=0, prefix="read"), Ts=(1, 2))
    # 6) non-default thresholds
    ref = make_reference(30_000, 1_500, seed=15)
    reads = make_reads(ref, 80, 150, seed=16, sub=0.05, ins=0.01, dele=0.01)
    e2e_case("params", fasta(ref), fasta(reads, width=0, prefix="read"), Ts=(1, 3),
             extra=("-evalue", "1e-10", "-coverage", "0.8", "-identity", "0.9", "-igap", "3", "-egap", "1"))
    # 7) records of exactly 2999/3000 bp and a 3001 bp record (fatal in the reference)
    x3000 = rand_seq(rng, 3000)
    x2999 = rand_seq(rng, 2999)
    reads = [mutate(rng, x3000[500:650], 0.01, 0, 0), mutate(rng, x2999[100:250], 0.01, 0, 0)]
    e2e_case("maxlen", fasta([x3000, x2999]), fasta(reads, width=0, prefix="read"), Ts=(1,))
    x3001 = rand_seq(rng, 3001)
    reads = [mutate(rng, x2999[10:160], 0.01, 0, 0), mutate(rng, x3001[10:160], 0.01, 0, 0),
             mutate(rng, x2999[300:450], 0.01, 0, 0)]
    e2e_case("toolong", fasta([x2999, x3001]), fasta(reads, width=0, prefix="read"), Ts=(1,))
    # 8) reads vs reads (C4 shape): both sides 150 bp
    ref = make_reference(50_000, 5_000, seed=17)
    a = make_reads(ref, 120, 150, seed=18)
    b = make_reads(ref, 120, 150, seed=19)
    e2e_case("reads_vs_reads", fasta(b, width=0, prefix="m2"), fasta(a, width=0, prefix="m1"))
    # 9) an empty query read placed at a chunk head for T=2 (ref UB: only T=1 recorded)
    ref = make_reference(10_000, 1_000, seed=20)
    reads = make_reads(ref, 10, 100, seed=21)
    reads[5] = ""
    e2e_case("empty_not_head", fasta(ref), fasta(reads, width=0, prefix="read"), Ts=(1, 3))


# ------------------------------------------------------------ revcomp ------
def gen_revcomp(rng):
    d = os.path.join(HERE, "revcomp")
    os.makedirs(d, exist_ok=True)
    cases = {
        "basic": b">r1 desc\nACGTNacgtu\nRY*-\r\nAC\n>r2\nGGGG\n>r3\n\n>r4\nUuTt\n",
        "crlf": b">a\r\nACGTT\r\nGG\r\n>b\r\nTTTT\r\n",
        "pre_text": b"junk before\n>x\nAC\n",
        "no_trailing_nl": b">x\nACGTA\n>y\nCCGT",
        "gt_in_header": b">x a>b\nACGT\n>y\nTT\n",
        "empty_header_only": b">only_header",
    }
    big = fasta(make_reference(30_000, 700, seed=22), width=61)
    cases["synthetic"] = big
    for name, data in cases.items():
        inp = os.path.join(d, name + ".in")
        outp = os.path.join(d, name + ".out")
        with open(inp, "wb") as f:
            f.write(data)
        subprocess.run([os.path.join(REF, "revComp"), inp, outp], check=True, stdout=subprocess.DEVNULL)
    print(f"revcomp: {len(cases)}")


def main():
    build_ref()
    rng = np.random.default_rng(20261015)
    gen_nw(rng)
    gen_ungapped(rng)
    gen_e2e(rng)
    gen_revcomp(rng)


if __name__ == "__main__":
    main()
