"""Canonical synthetic inputs.

numpy PCG64, iid uniform ACGT reference cut into fixed-length records;
"Illumina-like" reads: 90 % sampled uniformly from the reference
concatenation (record boundaries may be crossed) with 1 % substitutions (to a
different base), 0.05 % insertions, 0.05 % deletions; 10 % iid random reads.

Array forms return (seq: uint8[ACGT bytes], starts: uint64[n]) -- the exact
shape of the reference loaders' output (IMSAME.c:194-371) -- so large
workloads never go through Python strings.
"""
import numpy as np

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def make_reference_arr(total, rec_len, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    seq = ACGT[rng.integers(0, 4, total, dtype=np.uint8)]
    starts = np.arange(0, total, rec_len, dtype=np.uint64)
    return seq, starts


def make_reference(total, rec_len, seed):
    seq, starts = make_reference_arr(total, rec_len, seed)
    b = seq.tobytes().decode()
    return [b[s:s + rec_len] for s in starts.tolist()]


def _mutate_rows(rng, src, L, sub, ins, dele):
    """src: (n, L+pad) uint8 windows -> (n, L) reads with substitutions and
    (rare) indels; indel reads are re-built individually."""
    n, W = src.shape
    src = src.copy()
    # substitutions to a different base
    m = rng.random((n, W)) < sub
    if m.any():
        codes = np.searchsorted(ACGT, src[m])
        src[m] = ACGT[(codes + rng.integers(1, 4, codes.shape[0])) % 4]
    out = src[:, :L].copy()
    # indels: a deleted source base emits nothing, an insertion emits a random
    # base before its source base; rows are then cut to L (padded if short)
    ev = rng.random((n, W))
    rows = np.flatnonzero((ev < ins + dele).any(axis=1))
    if len(rows):
        e = ev[rows]
        keep = e >= dele
        insb = keep & (e < dele + ins)
        emit = keep.astype(np.int64) + insb
        pos = np.cumsum(emit, axis=1)                          # one past this base's slot
        buf = ACGT[rng.integers(0, 4, (len(rows), 2 * W + 1), dtype=np.uint8)]
        rr = np.broadcast_to(np.arange(len(rows))[:, None], e.shape)
        buf[rr[keep], (pos - 1)[keep]] = src[rows][keep]
        out[rows] = buf[:, :L]
    return out


def make_reads_arr(ref_seq, n, L, seed, sub=0.01, ins=0.0005, dele=0.0005, frac_true=0.9):
    """ref_seq: uint8 concatenation.  Returns (seq uint8[n*L], starts uint64[n])."""
    rng = np.random.Generator(np.random.PCG64(seed))
    pad = 8
    is_true = rng.random(n) < frac_true
    reads = np.empty((n, L), dtype=np.uint8)
    nt = int(is_true.sum())
    if nt:
        off = rng.integers(0, len(ref_seq) - (L + pad), nt)
        idx = off[:, None] + np.arange(L + pad)[None, :]
        reads[is_true] = _mutate_rows(rng, ref_seq[idx], L, sub, ins, dele)
    nr = n - nt
    if nr:
        reads[~is_true] = ACGT[rng.integers(0, 4, (nr, L), dtype=np.uint8)]
    starts = np.arange(0, n * L, L, dtype=np.uint64)
    return reads.reshape(-1), starts


def make_long_reads_arr(ref_seq, n, L, seed, sub=0.05, ins=0.025, dele=0.025, frac_true=0.9, chunk=1000):
    """C5's ONT-like long reads (5 % substitutions, 2.5 %
    insertions, 2.5 % deletions), generated `chunk` reads at a time so
    100k x 10 kbp stays within a few hundred MB of scratch.  Returns
    (seq uint8[n*L], starts uint64[n])."""
    rng = np.random.Generator(np.random.PCG64(seed))
    pad = int(L * dele * 1.5) + 64                    # deletions consume source bases
    out = np.empty((n, L), dtype=np.uint8)
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        is_true = rng.random(m) < frac_true
        blk = ACGT[rng.integers(0, 4, (m, L), dtype=np.uint8)]
        nt = int(is_true.sum())
        if nt:
            off = rng.integers(0, len(ref_seq) - (L + pad), nt)
            idx = off[:, None] + np.arange(L + pad)[None, :]
            blk[is_true] = _mutate_rows(rng, ref_seq[idx], L, sub, ins, dele)
        out[c0:c0 + m] = blk
    return out.reshape(-1), np.arange(0, n * L, L, dtype=np.uint64)


def make_reads(ref_records, n, L, seed, sub=0.01, ins=0.0005, dele=0.0005, frac_true=0.9):
    cat = np.frombuffer("".join(ref_records).encode(), dtype=np.uint8)
    seq, starts = make_reads_arr(cat, n, L, seed, sub, ins, dele, frac_true)
    b = seq.tobytes().decode()
    return [b[s:s + L] for s in starts.tolist()]


def to_fasta(seq, starts, prefix, width=80):
    """Array form -> FASTA bytes (LF, `>prefix_<i>` headers)."""
    b = seq.tobytes()
    ends = list(starts[1:].tolist()) + [len(b)]
    out = []
    for i, (s, e) in enumerate(zip(starts.tolist(), ends)):
        out.append(f">{prefix}_{i}\n".encode())
        if width:
            for k in range(s, e, width):
                out.append(b[k:min(e, k + width)] + b"\n")
        else:
            out.append(b[s:e] + b"\n")
    return b"".join(out)


def write_fasta(path, seq, starts, prefix, width=80):
    with open(path, "wb") as f:
        f.write(to_fasta(seq, starts, prefix, width))




def make_genome_pool(n_genomes, genome_bp, seed):
    """C4's shared pool: n iid uniform genomes."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return [ACGT[rng.integers(0, 4, genome_bp, dtype=np.uint8)] for _ in range(n_genomes)]


def make_metagenome_arr(pool, abundance, n, L, seed, sub=0.01, ins=0.0005, dele=0.0005, rc_frac=0.5):
    """n reads of length L drawn from the pool's genomes with the given
    abundance vector, Illumina-like errors, a fraction from the reverse
    strand.  Returns (seq uint8[n*L], starts uint64[n])."""
    rng = np.random.Generator(np.random.PCG64(seed))
    ab = np.asarray(abundance, dtype=np.float64)
    who = rng.choice(len(pool), size=n, p=ab / ab.sum())
    out = np.empty((n, L), np.uint8)
    for g in range(len(pool)):
        rows = np.flatnonzero(who == g)
        if not len(rows):
            continue
        s, _ = make_reads_arr(pool[g], len(rows), L, int(rng.integers(1 << 62)), sub, ins, dele, frac_true=1.0)
        s = s.reshape(len(rows), L)
        flip = rng.random(len(rows)) < rc_frac
        s[flip] = s[flip][:, ::-1]
        lut = np.zeros(256, np.uint8)
        lut[np.frombuffer(b"ACGT", np.uint8)] = np.frombuffer(b"TGCA", np.uint8)
        s[flip] = lut[s[flip]]
        out[rows] = s
    return out.reshape(-1), np.arange(0, n * L, L, dtype=np.uint64)


def adversarial_long_pairs():
    """Long pairs near the packed long kernel's size limit (nwp_fits: records
    and reads up to ~13.9 kbp at igap 5, egap 2) where its int16 frames are
    stressed most: scores climbing 4 per row over 12 kbp, tandem and
    dinucleotide repeats (long runs of equal maxima, ties in every column
    max), a 3 kbp deletion, homopolymer runs, a random pair (scores falling),
    and a read longer than its record."""
    rng = np.random.default_rng(77)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    rnd = lambda n: acgt[rng.integers(0, 4, n)]           # noqa: E731
    unit = rnd(37)
    x1 = rnd(13_900)
    rep = np.tile(unit, 376)[:13_900]
    ac = np.tile(np.frombuffer(b"AC", dtype=np.uint8), 6950)
    x4 = rnd(13_900)
    hp = np.concatenate([np.full(4000, ord("A"), np.uint8), rnd(5000), np.full(4900, ord("A"), np.uint8)])
    y7 = rnd(13_500)
    pairs = [
        (x1, x1[500:13_000]),                                             # identical 12.5 kbp
        (rep, rep[11:11 + 13_000]),                                       # tandem repeat, shifted
        (ac, np.concatenate([ac[:5000], rnd(1500), ac[:5000]])),          # dinucleotide + insertion
        (x4, np.concatenate([x4[:5000], x4[8000:]])),                     # 3 kbp deletion
        (hp, np.concatenate([np.full(3000, ord("A"), np.uint8), hp[4000:9000], np.full(3000, ord("A"), np.uint8)])),
        (rnd(13_900), rnd(12_000)),                                       # random: falling scores
        (y7[3000:9000].copy(), y7),                                       # read longer than its record
    ]
    return [x.tobytes() for x, _ in pairs], [y.tobytes() for _, y in pairs]
