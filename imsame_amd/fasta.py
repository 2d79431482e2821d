"""IMSAME's FASTA loading rules, vectorised (host side of the boundary).

Restates /root/reference/src/IMSAME.c:194-289 (database) and :320-371
(query), the same rules as the C loader of the CLI (csrc/host/fasta.c):

* a '>' opens a record (its start = bases loaded so far, :200) and the header
  runs to the next '\\n' (:212); text before the first '>' is ignored, and a
  '>' that is the file's very last byte opens nothing (:197);
* body bytes up to the next '>' are toupper()'d and only A/C/G/T are kept
  (:216-221, :343-346);
* database only: any other byte except '\\n' resets the running 12-mer
  (:229-231), as does every record start (:283).  Returned as the reset
  bitmap the device index takes (bit p = reset before base p).
"""
import numpy as np

_ACGT = np.zeros(256, dtype=bool)
_ACGT[np.frombuffer(b"ACGTacgt", dtype=np.uint8)] = True
_UPPER = np.arange(256, dtype=np.uint8)
_UPPER[ord("a"):ord("z") + 1] -= 32


def parse(data, want_brk=False):
    """bytes -> (seq uint8[ACGT], starts uint64[n], brk uint8 bitmap | None)."""
    b = np.frombuffer(data, dtype=np.uint8)
    n = len(b)
    gts = np.flatnonzero(b == ord(">"))
    if n and len(gts) and gts[-1] == n - 1:
        gts = gts[:-1]
    nls = np.append(np.flatnonzero(b == ord("\n")), n - 1)   # sentinel: EOF ends a header
    # header end (exclusive, after its '\n') of every '>'
    hend = nls[np.searchsorted(nls, gts)] + 1
    # record starts: a '>' inside a header opens nothing (chain over '>' bytes)
    recs = []
    nxt = 0
    for g, h in zip(gts.tolist(), hend.tolist()):
        if g >= nxt:
            recs.append((g, h))
            nxt = h
    body = np.zeros(n + 1, dtype=np.int8)
    if recs:
        rs = np.array(recs, dtype=np.int64)
        ends = np.append(rs[1:, 0], n)
        # mark body spans [hend, next record start) by a difference array
        np.add.at(body, rs[:, 1], 1)
        np.add.at(body, ends, -1)
    inbody = np.cumsum(body[:n]) > 0
    keep = inbody & _ACGT[b]
    seq = _UPPER[b[keep]]
    cum = np.concatenate(([0], np.cumsum(keep)))
    starts = cum[rs[:, 1]].astype(np.uint64) if recs else np.zeros(0, dtype=np.uint64)
    brk = None
    if want_brk:
        # reset events: body bytes that are neither ACGT nor '\n', plus record
        # starts; a kept base gets the bit if an event lies since the previous one
        ev = inbody & ~_ACGT[b] & (b != ord("\n"))
        evc = np.concatenate(([0], np.cumsum(ev)))
        kpos = np.flatnonzero(keep)
        prev = np.concatenate(([-1], kpos[:-1]))
        bit = evc[kpos] - evc[prev + 1] > 0
        bit |= np.isin(np.arange(len(kpos)), starts.astype(np.int64))
        # a record start with no base before the next record still resets: covered,
        # the next record's first base carries its own start bit
        brk = np.packbits(bit, bitorder="little") if len(kpos) else np.zeros(1, dtype=np.uint8)
    return seq, starts, brk


def load(path, want_brk=False):
    with open(path, "rb") as f:
        return parse(f.read(), want_brk)
