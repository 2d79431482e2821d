"""Readers for the committed golden vectors (tests/golden/, made by
tests/golden/make_golden.py from the compiled reference)."""
import gzip
import hashlib
import json
import os
import re

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
HEADER_RE = re.compile(rb"(\(\d+, \d+\) : \d+% \d+% \d+\n \$\$\$\$\$\$\$ \n)")
INFO_RE = re.compile(rb"^\[INFO\] (\d+ reads .*|The Jaccard-index is: .*)$", re.M)


def nw_pairs():
    with gzip.open(os.path.join(GOLDEN, "nw_pairs.jsonl.gz"), "rt") as f:
        return [json.loads(l) for l in f]


def ungapped_rows():
    with gzip.open(os.path.join(GOLDEN, "ungapped.jsonl.gz"), "rt") as f:
        rows = [json.loads(l) for l in f]
    cases = {}
    for c in sorted({r["case"] for r in rows}):
        with gzip.open(os.path.join(GOLDEN, f"ungapped_case{c}.json.gz"), "rt") as f:
            cases[c] = json.load(f)
    return rows, cases


def seqs_arrays(strs):
    cat = np.frombuffer("".join(strs).encode(), dtype=np.uint8).copy()
    starts = np.cumsum([0] + [len(s) for s in strs[:-1]]).astype(np.uint64)
    return cat, starts


def e2e_cases():
    d = os.path.join(GOLDEN, "e2e")
    return sorted(os.listdir(d))


def e2e_case(name):
    d = os.path.join(GOLDEN, "e2e", name)
    meta = json.load(open(os.path.join(d, "expected.json")))
    t1 = None
    p = os.path.join(d, "T1.align.gz")
    if os.path.exists(p):
        with gzip.open(p, "rb") as f:
            t1 = f.read()
    return dict(dir=d, db=os.path.join(d, "db.fa"), query=os.path.join(d, "query.fa"), meta=meta, t1=t1)


def record_multisets(blob):
    """Header and body multisets of an .align file.  With -n_threads > 1 the
    reference's header and body fprintf calls of different threads interleave
    (alignmentFunctions.c:167-168), but each call is atomic: drop the headers,
    and the remainder is a concatenation of bodies, each ending with the only
    empty line it contains (alignmentFunctions.c:270)."""
    heads = sorted(h.decode().split("\n")[0] + "\n" for h in HEADER_RE.findall(blob))
    rest = HEADER_RE.sub(b"", blob)
    bodies, pos = [], 0
    while pos < len(rest):
        e = rest.find(b"\n\n", pos)
        e = len(rest) if e < 0 else e + 2
        bodies.append(hashlib.sha1(rest[pos:e]).hexdigest())
        pos = e
    return heads, sorted(bodies)


def info_lines(stdout):
    return [m.decode() for m in INFO_RE.findall(stdout)]


def err_lines(stdout):
    return [l.decode() for l in stdout.split(b"\n") if l.startswith(b"ERR")]


def check_cli_against_golden(case, T, rc, stdout, align_blob):
    """Assert a CLI run (oracle or product) matches the reference's golden run."""
    exp = case["meta"]["runs"][str(T)]
    assert rc == exp["rc"], (rc, exp["rc"])
    assert err_lines(stdout) == exp["err"]
    assert info_lines(stdout) == exp["info"]
    if T == 1:
        assert align_blob == case["t1"]
    else:
        heads, bodies = record_multisets(align_blob)
        assert heads == exp["headers"]
        assert bodies == exp["body_sha1s"]
