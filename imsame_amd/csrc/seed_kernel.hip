// seed_kernel.hip -- per-read seed scan + ungapped extension + e-value test,
// and the per-round bookkeeping kernels.  Included by imsame_dev.hip (and by
// tests/emu/wave_emu.cpp under IMSAME_WAVE_EMU).
//
// Reference: computeAlignmentsByThread  alignmentFunctions.c:43-208
//            alignmentFromQuickHits     alignmentFunctions.c:276-387
// One thread per active read resumes the reference's visiting order
// (window-major, hits of a bucket in LIFO = descending-pos order) from the
// read's cursor and stops at the first hit whose e-value passes and whose
// record is not already known to be rejected for this read.
#include "wave_ops.h"

#define MEMO 16
#define NBUCKETS (1u << 24)
enum { RS_ACTIVE = 0, RS_DONE = 1, RS_ACCEPTED = 2, RS_ERROR = 3 };
// cursor of a read whose scan reached its last window (above every up_to):
// when its pending candidates are all rejected it is "not found" at once
// (update_one), instead of a next round whose scan finds nothing
#define CUR_EXHAUSTED (~1ull)

__device__ __forceinline__ uint32_t base2(uint32_t c) { return ((c >> 1) ^ (c >> 2)) & 3u; }  // A0 C1 G2 T3

struct SeedLaunch {
    const uint8_t *db; const uint64_t *db_start; uint64_t n_db, db_len;
    const uint8_t *q;  const uint64_t *q_start;  uint64_t n_q, q_len;
    const uint32_t *dbw, *qw;              // the same bases 2-bit packed (pk_base: word p >> 4 holds base p;
                                           // qw biased like q)
    const uint64_t *off; const uint2 *ent;        // CSR {pos - record start, record}, buckets in descending pos
    bool ent_abs = false;                  // ... {pos, record}: the absolute form (ent_pos)
    const uint32_t *active; uint32_t n_active;
    uint64_t read_from, rpt, T;
    uint64_t qs_lo, qs_lo_first;          // q_start holds reads >= qs_lo (a shard upload); reads
                                          // qs_lo_first .. qs_lo-1 are empty (see is_chunk_head)
    uint64_t *cur_p; uint32_t *cur_h; uint32_t *memo; uint8_t *nmemo; uint8_t *rstat;
    const uint64_t *minraw; uint32_t n_minraw;
    uint64_t max_rs; uint32_t short_ylen;
    uint64_t max_rec;                      // longest database record (a-priori rejection of whole reads)
    uint32_t spec;                         // candidates a read may emit this round (1..SPEC_MAX)
    uint32_t spec_weak;                    // ... a read with no rejection yet whose first candidate's hit
                                           // is weak (weak_hit): up to this many (<= 1: off)
    uint32_t budget;                       // ungapped extensions a read may run this round (0: no limit)
    uint32_t *next, *nnext;                // reads that paused on the budget (next round's active list)
    uint32_t *cbase, *ccnt;                // per read: first slot and count of this round's candidates
    uint32_t *perr;                        // per read: 1 + record of a pending size error, 0 = none
    const uint64_t *wcap;                  // per read: scan windows p < wcap[k] only (NULL: no cap;
                                           // database slices, imsame_dev_align_sliced)
    const uint64_t *wstart;                // per read: first window scanned >= wstart[k] (NULL: none)
    const uint32_t *minlen, *minident;     // acceptance tables of the launch (NULL: no a-priori rejection)
    uint32_t n_minlen, n_minident;
    uint32_t *cread, *csid, *ncand;        // class 0: ylen <= short_ylen
    int32_t *crow;                         // class 0: the record row of the read's first base by the
                                           // hit that made the candidate (INT32_MIN: none; NULL: off)
    bool weak_rows = false;                // ... for weak hits too (predicted_row)
    uint32_t *cread2, *csid2, *ncand2;     // class 1: longer reads
    unsigned long long *err;               // min (read << 32 | record)
    unsigned long long *nhits;
    // the scan's memory work (bench roofline of the seed stage, optional):
    // [0] windows probed (two CSR offsets each), [1] CSR entries read, [2]
    // 16-byte chunk pairs (database + query) loaded by ungapped extensions
    unsigned long long *nwork = nullptr;
    unsigned long long *dbg;               // diagnostics (IMSAME_DEBUG_ROUNDS): reads per scan outcome
                                           // (seed_outcome), NULL: off
};
// An index entry's database position (the reference's pos, one past the
// k-mer's last base, IMSAME.c:247) and its offset in the record.  The
// absolute form (databases below 2^32 bases, imsame_dev.hip:kmer_scatter)
// gives the position without the record's start, so a hit's first database
// words load while its record bounds are still in flight.
__device__ __forceinline__ int64_t ent_pos(const SeedLaunch &S, uint2 ent, int64_t xs) {
    return S.ent_abs ? (int64_t)ent.x : xs + (int64_t)ent.x;
}
__device__ __forceinline__ int64_t ent_rel(const SeedLaunch &S, uint2 ent, int64_t xs) {
    return S.ent_abs ? (int64_t)ent.x - xs : (int64_t)ent.x;
}
// ... the form fixed at compile time (the scan kernels: a select on the
// launch's flag would make the position wait for the record's start anyway)
template <bool ABS>
__device__ __forceinline__ int64_t ent_pos_t(uint2 ent, int64_t xs) { return ABS ? (int64_t)ent.x : xs + (int64_t)ent.x; }
template <bool ABS>
__device__ __forceinline__ int64_t ent_rel_t(uint2 ent, int64_t xs) { return ABS ? (int64_t)ent.x - xs : (int64_t)ent.x; }
// scan outcome classes of a read (diagnostics): no candidate + size error /
// paused / done; candidates + size error / paused / exhausted / spec full
#ifndef IMSAME_WAVE_EMU
__device__ __forceinline__ void seed_outcome(const SeedLaunch &S, uint32_t ne, bool perr, bool paused, bool exh) {
    if (!S.dbg) return;
    const int c = ne == 0 ? (perr ? 0 : paused ? 1 : 2) : (perr ? 3 : paused ? 4 : exh ? 5 : 6);
    atomicAdd(S.dbg + c, 1ull);
}
#endif
#define SPEC_MAX 8
// ... in rounds scanned by whole-wave groups (few reads: seed_group<64, SPEC_BIG>),
// so a random read with more than SPEC_MAX live e-value passes needs no
// extra round of one read (its NW alone is ~0.6 ms of a 2000-row record)
#define SPEC_BIG 32
// speculation width from a weak first candidate on (spec_after_first); 1 = off.
// 8: a read whose first e-value pass is weak (a random read's, by the idents
// quirk) emits up to 8 in round 1 instead of one -- C3 400.1 -> 393.6 ms (6
// rounds instead of 7, 2.85 NW per read instead of 2.88), C2 1/8 and 1/4
// shards 16.60 -> 16.34 and 30.08 -> 29.73 ms, C2 106.3 ms either way
// (profiles/r5q/, r5r/)
#ifndef SPEC_WEAK
#define SPEC_WEAK 8
#endif
// Hit budget per read and round: round 1 lets a read run SEED_BUDGET1
// ungapped extensions (true reads accept within a few), each later round 8x
// more, so reads that scan every window finish in a compacted list.
#define SEED_BUDGET1 32u
__host__ __device__ static inline uint32_t seed_budget(uint32_t b1, uint32_t round, uint32_t grow = 8) {
    if (b1 == 0) return 0;
    uint64_t b = b1;
    for (uint32_t k = 1; k < round && b < (1ull << 31); ++k) b *= grow;
    return b >= (1ull << 31) ? 0u : (uint32_t)b;
}

// 16 bytes p[a .. a+15] as 4 dwords (a >= 0; buffers carry >= 20 B of tail
// padding): one unaligned global_load_dwordx4 (the ROCm runtime runs the
// GPU in unaligned-access mode; hipcc emits the single load for this memcpy).
struct Bytes16 { uint32_t w[4]; };
__device__ __forceinline__ Bytes16 load16(const uint8_t *__restrict__ p, int64_t a) {
    Bytes16 r;
    __builtin_memcpy(&r, p + a, 16);
    return r;
}

// 2-bit packed bases (base2 codes A0 C1 G2 T3), 16 per dword: base p in word
// p >> 4, bits 2(p & 15).  The ungapped extension and the scan's k-mer codes
// read the database and the query in this form (imsame_dev.hip:pack2_kernel):
// 4 bytes per 16 bases instead of 16, so a 500 Mbp database (C3) is 125 MB and
// stays in the 256 MB Infinity Cache, and a 16-base chunk is a funnel shift of
// two dwords -- one new dword per chunk as a walk slides.  Both buffers hold
// only ACGT (the loaders drop every other byte, IMSAME.c:216-221, :340-345),
// so the codes lose nothing.  Arrays carry >= 2 words past their last base.
__device__ __forceinline__ uint32_t pk_base(const uint32_t *__restrict__ w, int64_t p) {
    return (w[p >> 4] >> (2u * (uint32_t)(p & 15))) & 3u;
}
// word w of the packed form of src (src[p] = base p, valid for lo <= p < hi;
// other slots 0): one 16-byte load where the word lies inside, four base2
// codes per dword gathered by shifts
__device__ __forceinline__ uint32_t pk_word(const uint8_t *__restrict__ src, int64_t w, int64_t lo, int64_t hi) {
    const int64_t p0 = w * 16;
    uint32_t v = 0;
    if (p0 >= lo && p0 + 16 <= hi) {
        const Bytes16 b = load16(src, p0);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t t = ((b.w[k] >> 1) ^ (b.w[k] >> 2)) & 0x03030303u;   // base2 of each byte
            const uint32_t u = t | (t >> 6);                                   // codes 0,1 -> bits 0-3; 2,3 -> 16-19
            v |= ((u & 0xFu) | ((u >> 12) & 0xF0u)) << (8 * k);
        }
    } else {
        for (int k = 0; k < 16; ++k) {
            const int64_t p = p0 + k;
            if (p >= lo && p < hi) v |= base2(src[p]) << (2 * k);
        }
    }
    return v;
}
// bit 2k set where slot k of a and b (bases) differ
__device__ __forceinline__ uint32_t pk_diff(uint32_t a, uint32_t b) {
    const uint32_t m = a ^ b;
    return (m | (m >> 1)) & 0x55555555u;
}
// the 12-mer code of bases p-11 .. p (first base most significant, as the
// index's kmer_code_kernel): slots 0..11 of one funnel shift, reversed in
// 2-bit groups (bit reverse, then swap each pair back)
__device__ __forceinline__ uint32_t kmer_code_pk(const uint32_t *__restrict__ w, int64_t p) {
    const int64_t a = p - (IMSAME_FIXED_K - 1);
    const uint32_t v = wv_alignbit(w[(a >> 4) + 1], w[a >> 4], 2u * (uint32_t)(a & 15));
    const uint32_t r = wv_bitrev(v);
    return (((r >> 1) & 0x55555555u) | ((r & 0x55555555u) << 1)) >> (32 - 2 * IMSAME_FIXED_K);
}

// Eight steps of the ungapped walk at once.  Each step of the reference's
// walk (alignmentFromQuickHits :321-337 right, :344-360 left) adds +-POINT to
// the score, counts an identity on a match, moves the best end when
// best <= score, and the walk stops after the step that takes the score to
// <= 0.  Over 8 steps whose match bits are m (bit j = step j) from a score of
// POINT*t, all of that is a function of (t, m) for t = 1..8 (t >= 9 cannot
// stop within 8 steps, so one row serves them all; row 0 = already stopped):
//   bits 0-3   js: the step the walk stops at, 8 = none
//   bits 4-8   mx + 8: the highest score (in POINTs, relative to the start)
//              of the steps before js (-8 if none)
//   bits 9-11  am: the LAST step reaching mx (ties move the end, :334)
//   bits 12-15 pc: identities up to js (all 8 steps when js = 8)
// The walk takes a table row per 8 bases instead of ~13 instructions and an
// exec-mask branch per base (the scan ran ~654 extensions per read at C3).
static_assert(IMSAME_POINT == 4, "ung_half scales t by POINT = 4");
struct UngTab { uint16_t v[10 * 256]; };
constexpr UngTab make_ung_tab() {
    UngTab T{};
    for (int t = 0; t < 10; ++t)
        for (int m = 0; m < 256; ++m) {
            int js = t ? 8 : 0, mx = -8, am = 0, pc = 0, s = 0;
            for (int j = 0; j < 8 && t; ++j) {
                const int eq = (m >> j) & 1;
                s += eq ? 1 : -1;
                pc += eq;
                if (t < 9 && t + s <= 0) { js = j; break; }
                if (mx <= s) { mx = s; am = j; }
            }
            T.v[t * 256 + m] = (uint16_t)(js | (mx + 8) << 4 | am << 9 | pc << 12);
        }
    return T;
}
__device__ constexpr UngTab g_ung_tab = make_ung_tab();
#define UNG_TAB_WORDS (10 * 256 / 2)
// a block's copy of the table in LDS (every thread of the block calls it)
__device__ __forceinline__ void ung_tab_load(uint16_t *lds) {
#ifndef IMSAME_WAVE_EMU
    const uint32_t *g = (const uint32_t *)g_ung_tab.v;
    for (uint32_t i = threadIdx.x; i < UNG_TAB_WORDS; i += blockDim.x) ((uint32_t *)lds)[i] = g[i];
    __syncthreads();
#endif
}
// one 8-step row: m8 = match bits, xr = the first step's position relative to
// the walk's origin, dir = +1 (right walk) / -1 (left walk)
__device__ __forceinline__ void ung_half(const uint16_t *__restrict__ tab, uint32_t m8, int &sc, int &best,
                                         int &endrel, uint32_t &idents, int xr, int dir) {
    const int t = min(max(sc, 0) >> 2, 9);
    const uint32_t e = tab[t * 256 + (int)m8];
    const int cand = sc + IMSAME_POINT * ((int)((e >> 4) & 31u) - 8);
    if (best <= cand) { best = cand; endrel = xr + dir * (int)((e >> 9) & 7u); }
    const uint32_t pc = e >> 12;
    idents += pc;
    sc = (e & 15u) < 8u ? 0 : sc + IMSAME_POINT * (2 * (int)pc - 8);
}
// 16 steps' match bits from pk_diff's mismatch bits (step k at bit 2k),
// steps >= n treated as mismatches: steps 0-7 in bits 0-7, 8-15 in bits 16-23
__device__ __forceinline__ uint32_t ung_match16(uint32_t mism, int64_t n) {
    uint32_t x = ~mism & (n >= 16 ? 0x55555555u : ((1u << (2 * (uint32_t)n)) - 1u) & 0x55555555u);
    x = (x | (x >> 1)) & 0x33333333u;
    x = (x | (x >> 2)) & 0x0F0F0F0Fu;
    return (x | (x >> 4)) & 0x00FF00FFu;
}

// The first chunk of each direction of a hit's extension (ungapped_raw):
// issued as soon as the hit's database position is known, before the
// record's bounds arrive (index entries in the absolute form, SeedLaunch::ent_abs)
struct UngFirst { uint32_t d0, d1, q0, q1, l0, l1, m0, m1; };
__device__ __forceinline__ UngFirst ung_first(const uint32_t *__restrict__ db, const uint32_t *__restrict__ q,
                                              int64_t pd0, int64_t pq0) {
    UngFirst f;
    f.d0 = db[pd0 >> 4]; f.d1 = db[(pd0 >> 4) + 1]; f.q0 = q[pq0 >> 4]; f.q1 = q[(pq0 >> 4) + 1];
    // left walk: chunk = bases x-15 .. x (x = bx0 = pd0 - 13 first); it needs
    // 15 bases below the start
    const int64_t bx0 = pd0 - IMSAME_FIXED_K - 1, by0 = pq0 - IMSAME_FIXED_K - 1;
    f.l0 = f.l1 = f.m0 = f.m1 = 0;
    if (bx0 >= 15 && by0 >= 15) {
        f.l0 = db[(bx0 - 15) >> 4]; f.l1 = db[((bx0 - 15) >> 4) + 1];
        f.m0 = q[(by0 - 15) >> 4]; f.m1 = q[((by0 - 15) >> 4) + 1];
    }
    return f;
}

// alignmentFromQuickHits (alignmentFunctions.c:276-387): the raw score in the
// reference's u64 wrap arithmetic (:373).  Loop bounds fold the reference's
// per-step tests (:321-322, :344-345) into one limit per direction.  The
// base-serial walk of the reference runs over 16-base chunks of the packed
// buffers (one dword load per chunk and side, the mismatches of 16 bases from
// one xor, two table rows per chunk: ung_half); the first chunk of each
// direction is fetched before either walk starts (f = ung_first(db, q, pd0,
// pq0)).  tab: g_ung_tab (its LDS copy in the scan kernels).
// (*nch, when given, counts the 16-base chunk pairs loaded)
__device__ __forceinline__ uint64_t ungapped_walk(const uint16_t *__restrict__ tab, const uint32_t *__restrict__ db,
                                                  const uint32_t *__restrict__ q, const UngFirst &f, int64_t pd0,
                                                  int64_t pq0, int64_t xs, int64_t xe, int64_t ys, int64_t ye,
                                                  int64_t dbl, int64_t ql, uint32_t *nch = nullptr) {
    int64_t end_x = pd0 - 1, beg_x = end_x - IMSAME_FIXED_K + 1;
    int sc = IMSAME_FIXED_K * IMSAME_POINT, best_r = sc, best_l = sc;
    uint32_t idents = IMSAME_FIXED_K;
    const int64_t bx0 = pd0 - IMSAME_FIXED_K - 1, by0 = pq0 - IMSAME_FIXED_K - 1;
    const bool lwin = bx0 >= 15 && by0 >= 15;
    // right walk: chunk = bases x .. x+15, words [x >> 4, (x >> 4) + 1];
    // word indices are recomputed from the positions (fewer live registers:
    // the scan kernels stay at 4 waves per SIMD, seed_group_kernel)
    const int64_t dq = pq0 - pd0;                        // y - x on the right walk
    const uint32_t dsh = 2u * (uint32_t)(pd0 & 15), qsh = 2u * (uint32_t)(pq0 & 15);
    uint32_t d0 = f.d0, d1 = f.d1, q0 = f.q0, q1 = f.q1;
    // left walk, downwards (slot 15 first); its shifts are the right walk's + 8 bases
    uint32_t l0 = f.l0, l1 = f.l1, m0 = f.m0, m1 = f.m1;
    const uint32_t lsh = (dsh + 8u) & 31u, lqsh = (qsh + 8u) & 31u;
    uint32_t nc = lwin ? 2 : 1;
    const int64_t fx = min(min(dbl - 1, xe), pd0 + (min(ql - 1, ye) - pq0));
    // (steps past n are mismatches to the table: they come after the last
    // real step, so they cannot move the best end, and the walk ends there)
    int er = -1;                        // end_x - pd0
    for (int64_t x = pd0; sc > 0 && x <= fx;) {
        const int64_t n = min((int64_t)16, fx - x + 1);
        const uint32_t m = ung_match16(pk_diff(wv_alignbit(d1, d0, dsh), wv_alignbit(q1, q0, qsh)), n);
        const int xr = (int)(x - pd0);
        ung_half(tab, m & 0xFFu, sc, best_r, er, idents, xr, 1);
        ung_half(tab, m >> 16, sc, best_r, er, idents, xr + 8, 1);
        x += n;                             // n < 16 only for the last chunk (x > fx after it)
        if (sc > 0 && x <= fx) { d0 = d1; d1 = db[(x >> 4) + 1]; q0 = q1; q1 = q[((x + dq) >> 4) + 1]; ++nc; }
    }
    end_x = pd0 + er;
    sc = best_r;                        // left pass restarts from the right max, best_l stays 48 (:339)
    const int64_t lx = max(max((int64_t)0, xs), bx0 - (by0 - max((int64_t)0, ys)));
    int64_t x = bx0, y = by0;
    if (lwin) {
        // a chunk's slot 15 - k is step k: bit-reversed, step k's mismatch bit lands at 2k
        int bl = 1;                     // beg_x - bx0
        while (sc > 0 && x >= lx && x >= 15 && y >= 15) {
            const int64_t n = min((int64_t)16, x - lx + 1);
            const uint32_t mism = wv_bitrev(pk_diff(wv_alignbit(l1, l0, lsh), wv_alignbit(m1, m0, lqsh))) >> 1;
            const uint32_t m = ung_match16(mism, n);
            const int xr = (int)(x - bx0);
            ung_half(tab, m & 0xFFu, sc, best_l, bl, idents, xr, -1);
            ung_half(tab, m >> 16, sc, best_l, bl, idents, xr - 8, -1);
            x -= n; y -= n;                 // n < 16 only when x passes lx (the loop ends)
            if (sc > 0 && x >= lx && x >= 15 && y >= 15) { l1 = l0; l0 = db[(x - 15) >> 4]; m1 = m0; m0 = q[(y - 15) >> 4]; ++nc; }
        }
        beg_x = bx0 + bl;
    }
    for (; sc > 0 && x >= lx; --x, --y) {                 // the first 15 bases of a buffer
        if (pk_base(db, x) == pk_base(q, y)) { sc += IMSAME_POINT; ++idents; } else sc -= IMSAME_POINT;
        if (best_l <= sc) { best_l = sc; beg_x = x; }
    }
    if (nch) *nch += nc;
    const uint64_t t_len = (uint64_t)(end_x - beg_x);
    return (uint64_t)idents * IMSAME_POINT - (t_len - idents) * IMSAME_POINT;
}
__device__ __forceinline__ uint64_t ungapped_raw(const uint16_t *__restrict__ tab, const uint32_t *__restrict__ db,
                                                 const uint32_t *__restrict__ q, int64_t pd0, int64_t pq0, int64_t xs,
                                                 int64_t xe, int64_t ys, int64_t ye, int64_t dbl, int64_t ql,
                                                 uint32_t *nch = nullptr) {
    return ungapped_walk(tab, db, q, ung_first(db, q, pd0, pq0), pd0, pq0, xs, xe, ys, ye, dbl, ql, nch);
}

// a thread's scan work: hits extended, and for the seed roofline windows
// probed, CSR entries read, extension chunk pairs loaded
struct SeedTally { uint64_t hits = 0, wins = 0, ents = 0; uint32_t chunks = 0; };

// Chunk heads (IMSAME.c:414,430-452): read r opens its
// chunk iff it starts where the chunk's first read from_c = i*floor(n/T)
// starts (empty reads in between hand the role on).  A shard upload holds the
// starts of reads >= qs_lo only; for from_c < qs_lo, q_start[from_c] == rs
// iff q_start[from_c] == q_start[qs_lo] (every read from_c .. qs_lo-1 empty,
// i.e. from_c >= qs_lo_first, computed on the host) and rs == q_start[qs_lo].
__device__ __forceinline__ bool is_chunk_head(const SeedLaunch &S, uint64_t r, uint64_t rs) {
    const uint64_t from_c = (S.rpt == 0) ? 0 : min(r / S.rpt, S.T - 1) * S.rpt;
    if (from_c >= S.qs_lo) return S.q_start[from_c] == rs;
    return from_c >= S.qs_lo_first && rs == S.q_start[S.qs_lo];
}

// NW(record, read) cannot be accepted, whatever its path: acceptance
// (alignmentFunctions.c:163) needs len >= minlen[ylen] and identities >=
// minident[len], minident is nondecreasing in len, and identities <=
// min(xlen, ylen) (build_alignment counts equal X/Y characters, each X and Y
// base at most once, :254-258).  Such a hit is rejected without running NW --
// the reference runs it and rejects it (C5: 10 kbp reads vs 2 kbp records).
// The test per read: NW(record, read) cannot be accepted iff
// accept_floor(S, ylen) > min(xlen, ylen) (the scans compute the floor once
// per read: two dependent table loads fewer per hit)
__device__ __forceinline__ uint64_t accept_floor(const SeedLaunch &S, uint64_t ylen) {
    if (!S.minlen || ylen >= S.n_minlen) return 0;
    uint32_t l0 = S.minlen[ylen];
    if (l0 == 0xFFFFFFFFu) return ~0ull;
    l0 = l0 ? l0 : 1u;                                    // minident[0] never passes
    if (l0 >= S.n_minident) return ~0ull;                 // longer than any path
    const uint32_t mi = S.minident[l0];
    return mi == 0xFFFFFFFFu ? ~0ull : (uint64_t)mi;
}
__device__ __forceinline__ bool nw_cannot_accept(uint64_t floor, uint64_t xlen, uint64_t ylen) {
    return floor > (xlen < ylen ? xlen : ylen);
}

// A hit whose record cannot be accepted for this read AND cannot trip the
// size abort (both lengths within max_read_size) has no observable effect
// whatever its e-value: the reference would extend it and either fail the
// e-value test or run an NW it then rejects.  Skipped before the extension.
__device__ __forceinline__ bool hit_irrelevant(const SeedLaunch &S, uint64_t floor, uint64_t xlen, uint64_t ylen) {
    return xlen <= S.max_rs && ylen <= S.max_rs && nw_cannot_accept(floor, xlen, ylen);
}
// ... and when even the longest record cannot accept the read, nothing the
// read's scan meets can: its outcome is "not found" without a scan.
__device__ __forceinline__ bool read_irrelevant(const SeedLaunch &S, uint64_t floor, uint64_t ylen) {
    return S.max_rec <= S.max_rs && hit_irrelevant(S, floor, S.max_rec, ylen);
}

// The first candidate of a read predicts its NW path (nw16_kernel.hip's
// first-sweep traceback window) when its hit is strong: an ungapped raw score
// of >= 7/3 per read base is a true hit's (C2: accepted first hits score
// 350-700, the e-value passes of random reads 236-350 by the idents quirk,
// Appendix A Q6).  A weak hit gets no prediction: its NW takes the second
// sweep, and it does not widen the window of the true hits' wave.
__device__ __forceinline__ bool weak_hit(uint64_t raw, uint64_t ylen) { return 3 * raw < 7 * ylen; }
__device__ __forceinline__ int32_t predicted_row(uint64_t raw, uint64_t ylen, int64_t rec_pos, int64_t read_pos,
                                                bool weak_rows = false) {
    return (!weak_rows && weak_hit(raw, ylen)) ? INT32_MIN : (int32_t)(rec_pos - read_pos);
}
// Speculation from the first candidate on: a read whose first e-value pass is
// weak (a random read's, by the idents quirk) will most likely see it
// rejected, and its next passes too, so it emits up to spec_weak of them in
// this round instead of one per round (exact for the same reason as any
// speculation: NW is pure, the first accepted in visiting order wins).
__device__ __forceinline__ uint32_t spec_after_first(const SeedLaunch &S, uint32_t spec, uint32_t nm, uint64_t raw,
                                                     uint64_t ylen) {
    return (nm == 0 && S.spec_weak > spec && weak_hit(raw, ylen)) ? S.spec_weak : spec;
}

template <bool ABS>
__device__ __forceinline__ void seed_one(const SeedLaunch &S, uint32_t idx, SeedTally &tl, const uint16_t *tab) {
    const uint64_t r = S.active[idx], k = r - S.read_from;
    const uint64_t rs = S.q_start[r], re = S.q_start[r + 1];
    const uint64_t ylen = re - rs;
    // chunk heads (IMSAME.c:414,430-452): a read borrows
    // the previous read's last base (the skip at :96-105 does not advance
    // curr_pos) unless it opens its chunk; an empty chunk-opening read (UB in
    // the reference) hands that role to the next read.
    const bool head = is_chunk_head(S, r, rs);
    const uint64_t p0 = rs - (head ? 0 : 1);
    uint64_t up_to = (r + 1 < S.n_q) ? (re ? re - 1 : 0) : S.q_len;          // :93
    if (S.wcap) up_to = min(up_to, S.wcap[k]);
    uint64_t p = S.cur_p[k];
    uint32_t h = S.cur_h[k];
    if (p == ~0ull) { p = p0 + IMSAME_FIXED_K - 1; h = 0; if (S.wstart) p = max(p, S.wstart[k]); }
    const uint32_t nm = S.nmemo[k];
    uint32_t memo[MEMO];
#pragma unroll
    for (int m = 0; m < MEMO; ++m) memo[m] = (m < (int)nm) ? S.memo[k * MEMO + m] : 0xFFFFFFFFu;
    const uint64_t mraw = ylen < S.n_minraw ? S.minraw[ylen] : ~0ull;
    const int64_t ys = (int64_t)rs, ye = (r == S.n_q - 1) ? (int64_t)S.q_len : (int64_t)re - 1;
    const uint64_t afl = accept_floor(S, ylen);
    if (read_irrelevant(S, afl, ylen)) { S.rstat[k] = RS_DONE; return; }      // nothing can be accepted
    // Up to `spec` e-value-passing hits of distinct, not-yet-rejected records,
    // in visiting order.  NW(record, read) is pure (Q18): whichever of them is
    // accepted first in this order is exactly the reference's accepted hit,
    // and a later hit of an emitted or rejected record cannot change that.
    uint32_t emit[SPEC_MAX];
    uint32_t ne = 0, perr = 0;
    int32_t row0 = INT32_MIN;              // first candidate's diagonal (nw16 traceback window)
    uint32_t code = 0;
    bool have = false, stop = false, paused = false;
    // A read that runs out of budget pauses at the hit it has not examined
    // and resumes there next round: the visiting order is unchanged, so this
    // only reshapes the work (reads that scan every window -- no true hit --
    // stop holding back the waves of reads that accept at their first hits).
    uint32_t budget = S.budget ? S.budget : 0xFFFFFFFFu;
    // speculate only for reads that already had a candidate rejected: a
    // read's first candidate is usually accepted (paused reads included)
    uint32_t spec = nm ? S.spec : 1u;
    for (; p < up_to && !stop; ++p, h = 0) {
        if (!have) {
            code = 0;
            for (int t = IMSAME_FIXED_K - 1; t >= 0; --t) code = (code << 2) | base2(S.q[p - t]);
            have = true;
        } else {
            code = ((code << 2) | base2(S.q[p])) & (NBUCKETS - 1);
        }
        const uint64_t lo = S.off[code], hi = S.off[code + 1];
        ++tl.wins;
        for (uint64_t e = lo + h; e < hi; ++e, ++h) {
            const uint2 ent = S.ent[e];
            ++tl.ents;
            const uint32_t sid = ent.y;
            bool skip = false;
#pragma unroll
            for (int m = 0; m < MEMO; ++m) skip |= memo[m] == sid;
            for (uint32_t m = 0; m < ne; ++m) skip |= emit[m] == sid;
            if (skip) continue;                 // NW(sid, r) already rejected or pending (Q18)
            if (hit_irrelevant(S, afl, S.db_start[sid + 1] - S.db_start[sid], ylen)) continue;
            if (budget == 0) {
                S.cur_p[k] = p; S.cur_h[k] = h;                      // resume at this hit
                paused = stop = true;
                break;
            }
            --budget;
            const int64_t xs = (int64_t)S.db_start[sid];
            const int64_t xe = (sid == S.n_db - 1) ? (int64_t)S.db_len : (int64_t)S.db_start[sid + 1] - 1;
            ++tl.hits;
            const uint64_t raw = ungapped_raw(tab, S.dbw, S.qw, ent_pos_t<ABS>(ent, xs), (int64_t)p + 1, xs, xe, ys, ye,
                                              (int64_t)S.db_len, (int64_t)S.q_len, &tl.chunks);
            if (mraw != ~0ull && raw >= mraw) {                      // e < min_e (:139)
                const uint64_t xlen = S.db_start[sid + 1] - S.db_start[sid];
                if (xlen > S.max_rs || ylen > S.max_rs) {            // terror (:155) if reached
                    perr = sid + 1;
                    stop = true;
                    break;
                }
                if (nw_cannot_accept(afl, xlen, ylen)) continue;     // NW would reject it
                if (ne == 0) {
                    row0 = predicted_row(raw, ylen, ent_rel_t<ABS>(ent, xs), (int64_t)(p + 1 - rs), S.weak_rows);
                    spec = spec_after_first(S, spec, nm, raw, ylen);
                }
                emit[ne++] = sid;
                if (ne == spec) {
                    S.cur_p[k] = p; S.cur_h[k] = h + 1;              // resume after this hit
                    stop = true;
                    break;
                }
            }
        }
        if (stop) break;
    }
#ifndef IMSAME_WAVE_EMU
    seed_outcome(S, ne, perr != 0, paused, ne < spec && !perr && !paused);
#endif
    if (ne == 0) {
        if (perr) {
            S.rstat[k] = RS_ERROR;
            wv_atomic_min64(S.err, (unsigned long long)((r << 32) | (perr - 1)));
        } else if (paused) {
            S.next[wv_atomic_add(S.nnext, 1u)] = (uint32_t)r;       // still active
        } else {
            S.rstat[k] = RS_DONE;
        }
        return;
    }
    if (ne < spec && !perr && !paused) { S.cur_p[k] = CUR_EXHAUSTED; S.cur_h[k] = 0; }   // scan exhausted
    S.perr[k] = perr;
    const bool shortc = ylen <= S.short_ylen;
    const uint32_t o = wv_atomic_add(shortc ? S.ncand : S.ncand2, ne);
    uint32_t *cr = shortc ? S.cread : S.cread2, *cs = shortc ? S.csid : S.csid2;
    for (uint32_t m = 0; m < ne; ++m) { cr[o + m] = (uint32_t)r; cs[o + m] = emit[m]; }
    if (shortc && S.crow)
        for (uint32_t m = 0; m < ne; ++m) S.crow[o + m] = m ? INT32_MIN : row0;
    S.cbase[k] = o; S.ccnt[k] = ne;
}

// ---------------------------------------------------------------------------
// Grouped scan for rounds with few active reads (latency-bound otherwise): a
// group of L lanes scans L consecutive windows of ONE read at a time, lane wl
// window p + wl in full (memory-level parallelism x L), each lane keeping the
// first `need` e-value-passing hits of its window that are not memo'd or
// already emitted.  The group then merges the lane lists in window order --
// exactly the single-lane visiting order -- with seed_one's semantics:
// distinct records up to `spec`, a size error stops the scan where it is
// reached, and the cursor lands right after the last consumed hit (a lane
// that stopped early because its list filled hands the rest of its window to
// the next round).  Pauses happen at window boundaries once the group has run
// `budget` extensions; like seed_one's pauses they only reshape the work.
// LDS: SEED_LDS_PER_LANE bytes per lane (the lane's list).
#define SEED_LDS_PER_LANE (SPEC_MAX * 8)
// ... and MEMO words per group after the lists (the read's memo, seed_group):
// a launch of L lanes per read and SM list entries per lane takes
// 256 * SM * 8 + (256 / L) * MEMO * 4 bytes of dynamic LDS per block
#define SEED_LDS_BLOCK(L, SM) (256 * (SM) * 8 + (256 / (L)) * MEMO * 4)
// list entry: {record, rank in the bucket | bit 31 size error | bit 30 weak hit}
#define LST_RANK 0x3FFFFFFFu
// lanes per read: enough lanes in flight to hide the probe latency
// (~1-4M lanes) without scanning many windows a read will not reach; nact =
// the reads the device scans at once (all lanes of a call)
__host__ __device__ static inline int seed_lanes(uint32_t nact) {
    return nact >= 2000000u ? 1 : nact >= 750000u ? 4 : 16;
}

// emit[] lives in registers, identical in every lane of the group (each lane
// runs the same merge); statically indexed so it never spills to scratch.
template <int SM>
__device__ __forceinline__ bool emit_has(const uint32_t (&em)[SM], uint32_t ne, uint32_t sid) {
    bool f = false;
#pragma unroll
    for (int m = 0; m < SM; ++m) f |= (uint32_t)m < ne && em[m] == sid;
    return f;
}

// (measured and dropped, round 6: C2 101.05-101.07 vs 101.10-101.17 ms, the 1/8
// shard 15.39 vs 15.37, C3 377.3 vs 376.5 -- the scan's bound is not the
// offsets' load, profiles/r6o/; off by default)
#ifndef SEED_PREFETCH
#define SEED_PREFETCH 0
#endif
// a record's bit in a read's memo filter (seed_group)
__device__ __forceinline__ uint32_t memo_bit(uint32_t sid) { return 1u << ((sid * 0x9E3779B1u) >> 27); }
// SM: the most candidates a read may emit (its list in LDS, emit[] in registers)
template <int L, int SM = SPEC_MAX, bool ABS = true>
__device__ void seed_group(const SeedLaunch &S, uint32_t gidx, int wl, int lane, uint2 *lst, SeedTally &tl,
                           const uint16_t *tab, uint32_t *gm) {
    const bool gvalid = gidx < S.n_active;
    const int gbase = lane - wl;                                  // first lane of the group
    uint64_t r = 0, k = 0, rs = 0, re = 0, ylen = 0, up_to = 0, p = 0;
    uint32_t h = 0, nm = 0, spec = 1, budget = 0xFFFFFFFFu;
    uint64_t mraw = ~0ull, afl = 0;
    int64_t ys = 0, ye = 0;
    if (gvalid) {
        r = S.active[gidx]; k = r - S.read_from;
        rs = S.q_start[r]; re = S.q_start[r + 1]; ylen = re - rs;
        const bool head = is_chunk_head(S, r, rs);                                   // chunk heads (Q4)
        const uint64_t p0 = rs - (head ? 0 : 1);
        up_to = (r + 1 < S.n_q) ? (re ? re - 1 : 0) : S.q_len;                     // :93
        if (S.wcap) up_to = min(up_to, S.wcap[k]);
        p = S.cur_p[k]; h = S.cur_h[k];
        if (p == ~0ull) { p = p0 + IMSAME_FIXED_K - 1; h = 0; if (S.wstart) p = max(p, S.wstart[k]); }
        nm = S.nmemo[k];
        spec = nm ? S.spec : 1u;
        budget = S.budget ? S.budget : 0xFFFFFFFFu;
        mraw = ylen < S.n_minraw ? S.minraw[ylen] : ~0ull;
        afl = accept_floor(S, ylen);
        ys = (int64_t)rs; ye = (r == S.n_q - 1) ? (int64_t)S.q_len : (int64_t)re - 1;
    }
    uint32_t emit[SM];
#pragma unroll
    for (int m = 0; m < SM; ++m) emit[m] = 0xFFFFFFFFu;
    // The read's rejected records (memo): copied once into the group's LDS
    // (gm, MEMO words) with a one-word filter of them, so an entry tests one
    // register bit, and the LDS copy only where the bit is set, instead of
    // nm dependent global loads per entry
    if (gvalid)
        for (uint32_t m = (uint32_t)wl; m < nm; m += L) gm[m] = S.memo[k * MEMO + m];
    wv_lds_sync();
    uint32_t mbloom = 0;
    for (uint32_t m = 0; m < nm; ++m) mbloom |= memo_bit(gm[m]);
    uint32_t ne = 0, perr = 0, used = 0;
    uint32_t e0p = 0, e0r = 0;             // first candidate's window (read-relative) and bucket rank
    bool done = !gvalid || p >= up_to || read_irrelevant(S, afl, ylen), paused = false,
         exhausted = gvalid && p >= up_to;
    // The CSR bounds of a lane's window are loaded one window ahead (SEED_PREFETCH):
    // the bucket offsets of the window the lane scans next (p + L + wl, if the
    // group advances) are in flight while the current window's entries and
    // extensions are walked, one dependent load fewer per window on the chain
    // offsets -> entries -> record bounds -> bases.
    uint64_t pf_lo = 0, pf_hi = 0;
    auto bounds = [&](const uint64_t w) {
        const uint32_t code = kmer_code_pk(S.qw, w);
        pf_lo = S.off[code]; pf_hi = S.off[code + 1];
    };
    if (SEED_PREFETCH && !done && p + (uint64_t)wl < up_to) bounds(p + (uint64_t)wl);
    while (wv_any(!done)) {
        // ---- every lane scans its window (no wave ops in here)
        const uint64_t pw = p + (uint64_t)wl;
        uint32_t nl = 0, last_rel = 0, ev = 0;
        bool full = false;
        uint64_t wbase = pf_lo, hi = pf_hi;
        if (SEED_PREFETCH && !done && pw + (uint64_t)L < up_to) bounds(pw + (uint64_t)L);
        if (!done && pw < up_to) {
            // (a read that may still start speculating lists for it already)
            const uint32_t need = (ne == 0 && nm == 0 && S.spec_weak > spec ? S.spec_weak : spec) - ne;
            if (!SEED_PREFETCH) {
                const uint32_t code = kmer_code_pk(S.qw, pw);
                wbase = S.off[code]; hi = S.off[code + 1];
            }
            ++tl.wins;
            // (the next entry is loaded while this one's extension runs)
            uint64_t e = wbase + (wl == 0 ? h : 0u);
            uint2 ent_nx = e < hi ? S.ent[e] : make_uint2(0u, 0u);
            for (; e < hi; ++e) {
                const uint2 ent = ent_nx;
                if (e + 1 < hi) ent_nx = S.ent[e + 1];
                ++tl.ents;
                const uint32_t sid = ent.y;
                bool skip = emit_has(emit, ne, sid);
                if (mbloom & memo_bit(sid))
                    for (uint32_t m = 0; m < nm; ++m) skip |= gm[m] == sid;
                for (uint32_t m = 0; m < nl; ++m) skip |= lst[m].x == sid;
                if (skip) continue;                       // NW(sid, r) rejected, pending or listed (Q18)
                const int64_t xs = (int64_t)S.db_start[sid], xn = (int64_t)S.db_start[sid + 1];
                const int64_t pd0 = ent_pos_t<ABS>(ent, xs);
                const UngFirst f = ung_first(S.dbw, S.qw, pd0, (int64_t)pw + 1);
                if (hit_irrelevant(S, afl, (uint64_t)(xn - xs), ylen)) continue;
                ++ev;
                const int64_t xe = (sid == S.n_db - 1) ? (int64_t)S.db_len : xn - 1;
                const uint64_t raw = ungapped_walk(tab, S.dbw, S.qw, f, pd0, (int64_t)pw + 1, xs, xe, ys, ye,
                                                   (int64_t)S.db_len, (int64_t)S.q_len, &tl.chunks);
                if (mraw != ~0ull && raw >= mraw) {                      // e < min_e (:139)
                    const uint64_t xlen = S.db_start[sid + 1] - S.db_start[sid];
                    const bool bad = xlen > S.max_rs || ylen > S.max_rs;   // terror (:155) if reached
                    if (!bad && nw_cannot_accept(afl, xlen, ylen)) continue; // NW would reject it
                    lst[nl++] = make_uint2(sid, (uint32_t)(e - wbase) | (bad ? 0x80000000u : 0u) |
                                                    (weak_hit(raw, ylen) ? 0x40000000u : 0u));
                    last_rel = (uint32_t)(e - wbase);
                    if (bad || nl == need) { full = true; break; }
                }
            }
        }
        tl.hits += ev;
        wv_lds_sync();                                    // lane lists written -> read by the group
        // ---- merge in window order (every lane of the group runs the same merge)
        uint32_t tot = 0;
        bool stop = done;
        for (int wk = 0; wk < L; ++wk) {
            const uint32_t cnt = (uint32_t)wv_shfl((int)nl, gbase + wk);
            const bool fullk = wv_shfl((int)full, gbase + wk) != 0;
            const uint32_t lastk = (uint32_t)wv_shfl((int)last_rel, gbase + wk);
            tot += (uint32_t)wv_shfl((int)ev, gbase + wk);
            if (stop) continue;
            const uint64_t pk = p + (uint64_t)wk;
            if (pk >= up_to) { exhausted = true; stop = true; continue; }
            const uint2 *lk = lst + (wk - wl) * SM;                 // lane wk's list
            for (uint32_t m = 0; m < cnt && !stop; ++m) {
                const uint2 it = lk[m];
                if (emit_has(emit, ne, it.x)) continue;            // emitted by an earlier window
                if (it.y & 0x80000000u) { perr = it.x + 1; stop = true; break; }
                if (ne == 0) {
                    e0p = (uint32_t)(pk - rs); e0r = it.y & LST_RANK;
                    if (nm == 0 && S.spec_weak > spec && (it.y & 0x40000000u)) spec = S.spec_weak;   // spec_after_first
                }
#pragma unroll
                for (int q2 = 0; q2 < SM; ++q2) emit[q2] = ((uint32_t)q2 == ne) ? it.x : emit[q2];
                ++ne;
                if (ne == spec) {                                  // resume after this hit
                    if (wl == 0) { S.cur_p[k] = pk; S.cur_h[k] = (it.y & LST_RANK) + 1; }
                    stop = true;
                }
            }
            if (!stop && fullk) {                                  // lane list ran dry mid-window
                if (wl == 0) { S.cur_p[k] = pk; S.cur_h[k] = lastk + 1; }
                paused = true; stop = true;
            }
        }
        if (!stop) {
            p += L; h = 0; used += tot;
            if (p >= up_to) { exhausted = true; stop = true; }
            else if (used >= budget) {
                if (wl == 0) { S.cur_p[k] = p; S.cur_h[k] = 0; }
                paused = true; stop = true;
            }
        }
        done = stop;
        wv_lds_sync();                                    // lists read before the next scan rewrites them
    }
    if (!gvalid || wl != 0) return;
#ifndef IMSAME_WAVE_EMU
    seed_outcome(S, ne, perr != 0, paused, exhausted);
#endif
    if (ne == 0) {
        if (perr) {
            S.rstat[k] = RS_ERROR;
            wv_atomic_min64(S.err, (unsigned long long)((r << 32) | (perr - 1)));
        } else if (paused) {
            S.next[wv_atomic_add(S.nnext, 1u)] = (uint32_t)r;       // still active
        } else {
            S.rstat[k] = RS_DONE;
        }
        return;
    }
    if (exhausted && !perr) { S.cur_p[k] = CUR_EXHAUSTED; S.cur_h[k] = 0; }   // scan exhausted
    S.perr[k] = perr;
    const bool shortc = ylen <= S.short_ylen;
    const uint32_t o = wv_atomic_add(shortc ? S.ncand : S.ncand2, ne);
    uint32_t *cr = shortc ? S.cread : S.cread2, *cs = shortc ? S.csid : S.csid2;
#pragma unroll
    for (int m = 0; m < SM; ++m)
        if ((uint32_t)m < ne) { cr[o + m] = (uint32_t)r; cs[o + m] = emit[m]; }
    if (shortc && S.crow) {
        // the first candidate's hit again: its entry gives the record position
        // and its extension the strength
        const uint2 ent = S.ent[S.off[kmer_code_pk(S.qw, rs + e0p)] + e0r];
        const int64_t xs = (int64_t)S.db_start[ent.y];
        const int64_t xe = (ent.y == S.n_db - 1) ? (int64_t)S.db_len : (int64_t)S.db_start[ent.y + 1] - 1;
        const uint64_t raw = ungapped_raw(tab, S.dbw, S.qw, ent_pos_t<ABS>(ent, xs), (int64_t)(rs + e0p) + 1, xs, xe, ys,
                                          ye, (int64_t)S.db_len, (int64_t)S.q_len);
        S.crow[o] = predicted_row(raw, ylen, ent_rel_t<ABS>(ent, xs), (int64_t)e0p + 1, S.weak_rows);
        for (uint32_t m = 1; m < ne; ++m) S.crow[o + m] = INT32_MIN;
    }
    S.cbase[k] = o; S.ccnt[k] = ne;
}

// Database slices (imsame_dev_align_sliced): the window of each accepted
// read's hit.  The accepted record s is the first whose NW accepted, and NW
// is pure (Q18), so its hit is the FIRST e-value-passing hit of s in
// visiting order: rescan the read's windows for it (read-start logic as
// seed_one; usually the first window).
__device__ __forceinline__ void accept_window_one(const SeedLaunch &S, const imsame_read_result *res, uint32_t k,
                                                  uint64_t *wout) {
    if (res[k].status != 1) return;
    const uint64_t r = S.read_from + k;
    const uint64_t rs = S.q_start[r], re = S.q_start[r + 1], ylen = re - rs;
    const bool head = is_chunk_head(S, r, rs);
    const uint64_t p0 = rs - (head ? 0 : 1);
    uint64_t up_to = (r + 1 < S.n_q) ? (re ? re - 1 : 0) : S.q_len;
    if (S.wcap) up_to = min(up_to, S.wcap[k]);
    const uint64_t mraw = ylen < S.n_minraw ? S.minraw[ylen] : ~0ull;
    const int64_t ys = (int64_t)rs, ye = (r == S.n_q - 1) ? (int64_t)S.q_len : (int64_t)re - 1;
    const uint32_t sid = (uint32_t)res[k].db_seq;
    const int64_t xs = (int64_t)S.db_start[sid];
    const int64_t xe = (sid == S.n_db - 1) ? (int64_t)S.db_len : (int64_t)S.db_start[sid + 1] - 1;
    uint64_t w = ~0ull;
    for (uint64_t p = p0 + IMSAME_FIXED_K - 1; p < up_to && w == ~0ull; ++p) {
        const uint32_t code = kmer_code_pk(S.qw, p);
        for (uint64_t e = S.off[code]; e < S.off[code + 1]; ++e) {
            const uint2 ent = S.ent[e];
            if (ent.y != sid) continue;
            const uint64_t raw = ungapped_raw(g_ung_tab.v, S.dbw, S.qw, ent_pos(S, ent, xs), (int64_t)p + 1, xs, xe, ys, ye,
                                              (int64_t)S.db_len, (int64_t)S.q_len);
            if (mraw != ~0ull && raw >= mraw) { w = p; break; }
        }
    }
    wout[k] = w;
}

struct UpdLaunch {
    const uint32_t *cread, *csid; uint32_t n;
    const imsame_read_result *out;
    uint64_t read_from;
    imsame_read_result *res;
    uint8_t *rstat; uint32_t *memo; uint8_t *nmemo;
    const uint32_t *cbase, *ccnt, *perr;
    const uint64_t *cur_p;                 // CUR_EXHAUSTED: nothing left to scan
    uint32_t *next; uint32_t *nnext;
    unsigned long long *cells; unsigned long long *nacc;
    unsigned long long *err;
    const uint64_t *db_start;
    const uint64_t *flags = nullptr;       // NW launch flags (C_FLAGS): bit 2 = a wave ran no task
    unsigned long long *waste = nullptr;   // candidates computed past a read's accepted one (speculation)
    const uint32_t *perm = nullptr;        // the candidates are perm[0 .. n) (NULL: 0 .. n); whole reads'
                                           // sets (imsame_dev.hip: the round-1 launch cut in two)
};

// Per read (run by its first candidate): the first accepted candidate in
// visiting order is the read's result (NWaligned = 1, :172); rejected ones
// before it are remembered; none accepted -> a pending size error fires
// (terror, :155) or the read continues from its cursor next round.
__device__ __forceinline__ void update_one(const UpdLaunch &U, uint32_t c, uint64_t &cells, uint64_t &acc,
                                           uint64_t &waste) {
    const uint32_t r = U.cread[c];
    const uint64_t k = r - U.read_from;
    const imsame_read_result oc = U.out[c];
    cells += (uint64_t)(U.db_start[oc.db_seq + 1] - U.db_start[oc.db_seq]) * oc.ylen;
    const uint32_t base = U.cbase[k];
    if (c != base) return;
    const uint32_t cnt = U.ccnt[k];
    uint32_t nm = U.nmemo[k];
    for (uint32_t m = 0; m < cnt; ++m) {
        const imsame_read_result o = U.out[base + m];
        if (o.status == 1) {
            U.res[k] = o;
            U.rstat[k] = RS_ACCEPTED;
            acc += 1;
            waste += cnt - m - 1;                          // speculative NWs past the accepted one
            U.nmemo[k] = (uint8_t)nm;
            return;
        }
        if (nm < MEMO) U.memo[k * MEMO + nm++] = (uint32_t)o.db_seq;
    }
    U.nmemo[k] = (uint8_t)nm;
    if (U.perr[k]) {
        U.rstat[k] = RS_ERROR;
        wv_atomic_min64(U.err, (unsigned long long)(((uint64_t)r << 32) | (U.perr[k] - 1)));
        return;
    }
    if (U.cur_p[k] == CUR_EXHAUSTED) { U.rstat[k] = RS_DONE; return; }      // no hit left: not found
    U.next[wv_atomic_add(U.nnext, 1u)] = r;
}

struct InitLaunch {
    const uint64_t *q_start; uint64_t read_from; uint32_t n;
    imsame_read_result *res; uint64_t *cur_p; uint32_t *cur_h; uint8_t *nmemo; uint8_t *rstat;
    uint32_t *active;
};

__device__ __forceinline__ void init_one(const InitLaunch &I, uint32_t k) {
    const uint64_t r = I.read_from + k;
    imsame_read_result z;
    memset(&z, 0, sizeof z);
    z.ylen = (uint32_t)(I.q_start[r + 1] - I.q_start[r]);
    I.res[k] = z;
    I.cur_p[k] = ~0ull; I.cur_h[k] = 0; I.nmemo[k] = 0; I.rstat[k] = RS_ACTIVE;
    I.active[k] = (uint32_t)r;
}

#ifndef IMSAME_WAVE_EMU
// the wave's tallies summed first: one atomic per counter per wave (every
// lane of the wave reaches this)
__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned lo = (unsigned)__shfl_xor((int)(unsigned)v, o), hi = (unsigned)__shfl_xor((int)(unsigned)(v >> 32), o);
        v += ((unsigned long long)hi << 32) | lo;
    }
    return v;
}
__device__ __forceinline__ void seed_tally_flush(const SeedLaunch &S, const SeedTally &tl) {
    const unsigned long long h = wave_sum64(tl.hits);
    const bool lead = (threadIdx.x & 63) == 0;
    if (lead && h) atomicAdd(S.nhits, h);
    if (S.nwork) {
        const unsigned long long w = wave_sum64(tl.wins), e = wave_sum64(tl.ents), c = wave_sum64(tl.chunks);
        if (lead && w) { atomicAdd(S.nwork, w); atomicAdd(S.nwork + 1, e); atomicAdd(S.nwork + 2, c); }
    }
}
__global__ void accept_window_kernel(const SeedLaunch S, const imsame_read_result *res, uint32_t n, uint64_t *wout) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) accept_window_one(S, res, k, wout);
}
// <= 128 VGPRs (4 waves per SIMD): the scans of later rounds and of round 1b
// run beside NW launches, whose 19-column waves hold 256 VGPRs each, so a
// SIMD with one NW wave has 256 left -- two scan waves at 128, one at 136.  A
// scan kernel compiled to 135 VGPRs ran round 1b's scans 2.8x longer next to
// NW (C2 1/8 shard 3.1 -> 8.8 ms, profiles/r5f/).  (The whole-wave groups with
// SPEC_BIG candidates in registers would spill at 128; they run the small
// later rounds.)
#ifndef SEED_WAVES_PER_EU
#define SEED_WAVES_PER_EU 4
#endif
// Wave-stride over the groups (a launch may hold fewer waves than groups,
// imsame_dev.hip:seed_blocks; a wave's groups are consecutive, so the loop's
// exit is wave-uniform)
template <int L, int SM = SPEC_MAX, bool ABS = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SM > SPEC_MAX ? 1 : SEED_WAVES_PER_EU)))
void seed_group_kernel(SeedLaunch S) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63, wl = lane % L;
    uint2 *lst = (uint2 *)smem + threadIdx.x * SM;
    uint32_t *gm = (uint32_t *)(smem + 256 * SM * 8) + (threadIdx.x / L) * MEMO;   // SEED_LDS_GROUP
    __shared__ uint16_t tab[10 * 256];
    ung_tab_load(tab);
    constexpr uint32_t GPW = 64 / L;                       // groups per wave
    const uint32_t nwv = gridDim.x * (blockDim.x >> 6);
    SeedTally tl;
    for (uint32_t wv = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); (uint64_t)wv * GPW < S.n_active; wv += nwv)
        seed_group<L, SM, ABS>(S, wv * GPW + (uint32_t)lane / L, wl, lane, lst, tl, tab, gm);
    seed_tally_flush(S, tl);
}

template <bool ABS = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SEED_WAVES_PER_EU))) void seed_kernel(SeedLaunch S) {
    __shared__ uint16_t tab[10 * 256];
    ung_tab_load(tab);
    SeedTally tl;
    for (uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x; idx < S.n_active; idx += gridDim.x * blockDim.x)
        seed_one<ABS>(S, idx, tl, tab);
    seed_tally_flush(S, tl);
}

// Grid-stride over the candidates: the host launches few waves (imsame_dev.hip:
// upd_blocks).  A round's update is queued behind its NW launch while other
// lanes' NW waves hold the chip; every wave it launches must win a slot
// freed by one of those waves (each runs ~ms), so one wave per 64 candidates
// -- 4.6k waves at C2's round 1 -- waited ~10 ms (profiles/r5end4/ C2
// timeline: lane 2's round 1 ended at 79.8 ms, its round-2 scan began 90.7).
__global__ void update_kernel(UpdLaunch U) {
    uint64_t cells = 0, acc = 0, waste = 0;
    // a non-persistent NW wave that found no arena slot left its candidates'
    // rows unwritten: consume none of them (the host fails the call)
    if (U.flags && (__hip_atomic_load(U.flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 4u)) return;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < U.n; c += gridDim.x * blockDim.x)
        update_one(U, U.perm ? U.perm[c] : c, cells, acc, waste);
    if (cells) atomicAdd(U.cells, (unsigned long long)cells);
    if (waste && U.waste) atomicAdd(U.waste, (unsigned long long)waste);
    if (acc) atomicAdd(U.nacc, (unsigned long long)acc);
}

__global__ void init_kernel(InitLaunch I) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < I.n) init_one(I, k);
}
#endif
