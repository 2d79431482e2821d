"""Window parity of a large device run against the oracle -- TEST
INFRASTRUCTURE (tests/, and bench.py's cpu_baseline leg as the checker).

The oracle (oracle/imsame_oracle.c) aligns only the reads of a few windows of
the WHOLE query (its -n_threads chunk heads), so a 1M-read device result can
be checked read for read at start, middle (across a chunk head) and end in
seconds.  Reference: computeAlignmentsByThread, alignmentFunctions.c:43-208.
"""
import numpy as np

from imsame_amd import PARITY_FIELDS


def windows(lo, hi, n_total, n_threads=16, w=1500):
    """[start, middle, end) windows of reads [lo, hi) of an n_total-read
    query: the middle one straddles a chunk head {k * floor(n/T)} inside the
    range when there is one (a head reads no borrowed base)."""
    w = min(w, max((hi - lo) // 3, 1))
    rpt = n_total // max(n_threads, 1)
    heads = [k * rpt for k in range(1, n_threads) if rpt and lo + w // 2 <= k * rpt <= hi - w // 2]
    mid = heads[len(heads) // 2] if heads else (lo + hi) // 2
    out = [(lo, lo + w), (mid - w // 2, mid - w // 2 + w), (hi - w, hi)]
    return sorted(set((max(lo, a), min(hi, b)) for a, b in out))


def check_windows(oracle, ref, rst, q, qs, res, res_lo, wins, n_threads, params=None, count_ref=False):
    """Compare res (rows of reads res_lo, res_lo + 1, ...) with the oracle on
    the windows; the oracle's memo of rejected pairs (identical results, NW is
    pure: Appendix A Q18) keeps it fast.  It also counts the NW calls on the
    windows: `nw_distinct` with the memo (the distinct (read, record) pairs up
    to each read's accepted one -- the device computes exactly these plus its
    speculation) and, with count_ref, `nw_reference` without it (the
    reference's own count: it re-runs NW at every e-value-passing hit of a
    rejected record, alignmentFunctions.c:126-186)."""
    import ctypes as C
    oracle.lib.or_last_nw.restype = C.c_uint64
    oracle.lib.or_set_memo_rejected(1)
    try:
        rc, exp, er = oracle.align_windows(ref, rst, q, qs, wins, params, n_threads)
        nw_distinct = int(oracle.lib.or_last_nw())
    finally:
        oracle.lib.or_set_memo_rejected(0)
    nw_ref = None
    if count_ref:
        rc2, exp2, _ = oracle.align_windows(ref, rst, q, qs, wins, params, n_threads)
        nw_ref = int(oracle.lib.or_last_nw())
        assert rc2 == rc and all(np.array_equal(a[f], b[f]) for a, b in zip(exp, exp2) for f in PARITY_FIELDS)
    compared = identical = 0
    bad = []
    for (a, b), e in zip(wins, exp):
        got = res[a - res_lo:b - res_lo]
        same = np.all([got[f] == e[f] for f in PARITY_FIELDS], axis=0)
        compared += b - a
        identical += int(same.sum())
        bad += [a + int(i) for i in np.flatnonzero(~same)[:3]]
    return {"reads_compared": compared, "identical": identical, "windows": [list(x) for x in wins],
            "n_threads": n_threads, "oracle_rc": int(rc), "first_mismatches": bad,
            "accepted_in_windows": int(sum(int((res[a - res_lo:b - res_lo]["status"] == 1).sum()) for a, b in wins)),
            "oracle_nw_distinct": nw_distinct, "oracle_nw_reference": nw_ref}


def chunk_slices(n_total, n_threads, parts):
    """Every read of an n_total-read query, as `parts` calls of n_threads
    windows each: call p holds the p-th of `parts` slices of every -n_threads
    chunk [t*floor(n/T), (t+1)*floor(n/T)) (the last chunk runs to the end), so
    each oracle call keeps one thread per chunk busy (IMSAME.c:414,430-452)."""
    T = max(n_threads, 1)
    rpt = n_total // T
    bounds = [(t * rpt, n_total if t == T - 1 else (t + 1) * rpt) for t in range(T)] if rpt else [(0, n_total)]
    calls = []
    for p in range(parts):
        wins = []
        for f, e in bounds:
            a, b = f + (e - f) * p // parts, f + (e - f) * (p + 1) // parts
            if b > a:
                wins.append((a, b))
        calls.append(wins)
    return calls


def check_all(oracle, ref, rst, q, qs, res, n_threads, parts=4, params=None, progress=None):
    """EVERY read of the query against the oracle (its memo of rejected
    pairs on, as check_windows): `parts` oracle calls of n_threads windows
    (chunk_slices), each followed by a progress callback."""
    tot = {"reads_compared": 0, "identical": 0, "first_mismatches": [], "oracle_rc": 0, "parts": parts,
           "n_threads": n_threads}
    for k, wins in enumerate(chunk_slices(len(qs), n_threads, parts)):
        out = check_windows(oracle, ref, rst, q, qs, res, 0, wins, n_threads, params)
        tot["reads_compared"] += out["reads_compared"]
        tot["identical"] += out["identical"]
        tot["first_mismatches"] += out["first_mismatches"][:3]
        tot["oracle_rc"] = tot["oracle_rc"] or out["oracle_rc"]
        if progress:
            progress(k + 1, parts, tot)
    return tot
