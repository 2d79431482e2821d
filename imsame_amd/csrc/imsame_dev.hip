// imsame_dev.hip -- MI355X (gfx950) implementation of include/imsame_dev.h.
//
// Device pipeline for one imsame_dev_align call:
//   index  : kmer_code -> count -> scan -> scatter -> segsort   (CSR in HBM)
//   rounds : seed_kernel   first e-value-passing, not-yet-rejected hit per
//                          active read, in the reference's visiting order
//            nw_kernel     gapped alignment + backtrack + accept (wavefront)
//            update_kernel accepted -> result; rejected -> memo + next round
// The reference visits (window, hit) pairs in order and stops at the first
// accepted one (alignmentFunctions.c:91-195).  NW is a pure function of
// (record, read), so a rejected record is skipped
// on later hits instead of being recomputed; results are unchanged.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <limits.h>
#include <time.h>
#include <sched.h>
#include <vector>
#include <algorithm>
#include <thread>
#include <mutex>
#include <condition_variable>
#include "../../include/imsame_dev.h"

#include "tables.h"
#include "nw_kernel.hip"
#include "nw16_kernel.hip"
#include "nwl_kernel.hip"
#include "nwp_kernel.hip"
#include "seed_kernel.hip"
#include "round_policy.h"


#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "[imsame] HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
    return IMSAME_E_HIP; } } while (0)

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------

// ---------------------------------------------------------------------------
// index build (replaces IMSAME.c:232-281)
// ---------------------------------------------------------------------------
__global__ void mark_record_starts(const uint64_t *st, uint64_t n, uint64_t L, uint32_t *brk) {
    uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (k < n && st[k] < L) atomicOr(&brk[st[k] >> 5], 1u << (st[k] & 31));
}

// Grid-stride loops: a dispatch holds < 2^32 work-items, a database may
// hold more bases.
#define GRID_STRIDE(p, n) \
    for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p < (n); p += (uint64_t)gridDim.x * blockDim.x)

// the 2-bit packed bases (seed_kernel.hip:pk_word): words [w0, w1) of dst
// (biased: dst[w] holds bases 16w ..) from src (biased: src[p] = base p,
// valid for lo <= p < hi; other slots 0)
// ... and, where `bad` is given, bit 0 of *bad set if a byte of [lo, hi) in
// these words is not 'A', 'C', 'G' or 'T': the 2-bit codes (and nw16's
// base_code) alias every other byte to one of them, so the bases must be what
// IMSAME's loaders keep (IMSAME.c:216-221, :340-345; include/imsame_dev.h)
__device__ __forceinline__ bool acgt_word_bad(const uint8_t *src, int64_t w, int64_t lo, int64_t hi) {
    bool bad = false;
    for (int64_t p = max(w * 16, lo), e = min(w * 16 + 16, hi); p < e; ++p) {
        const uint8_t b = src[p];
        bad |= b != 'A' && b != 'C' && b != 'G' && b != 'T';
    }
    return bad;
}
// (the check stops at bad_hi: an upload's 64 zero bytes past its last read
// are packed, not checked)
__global__ void pack2_kernel(const uint8_t *src, int64_t lo, int64_t hi, uint32_t *dst, uint64_t w0, uint64_t w1,
                             unsigned long long *bad = nullptr, int64_t bad_hi = INT64_MAX) {
    bool b = false;
    GRID_STRIDE(k, w1 - w0) {
        dst[w0 + k] = pk_word(src, (int64_t)(w0 + k), lo, hi);
        if (bad) b |= acgt_word_bad(src, (int64_t)(w0 + k), lo, min(hi, bad_hi));
    }
    if (b) atomicOr(bad, 8ull);
}

// code of the 12-mer ending at base p, or ~0 when a reset lies in (p-11, p]
__global__ void kmer_code_kernel(const uint8_t *seq, uint64_t L, const uint32_t *brk, uint32_t *codes,
                                 uint32_t *cnt) {
    GRID_STRIDE(p, L) {
        uint32_t code = 0xFFFFFFFFu;
        if (p >= IMSAME_FIXED_K - 1) {
            const uint64_t b0 = p - (IMSAME_FIXED_K - 2);           // bits p-10 .. p
            const uint64_t w = b0 >> 5;
            const uint64_t win = ((uint64_t)brk[w] | ((uint64_t)brk[w + 1] << 32)) >> (b0 & 31);
            if ((win & ((1u << (IMSAME_FIXED_K - 1)) - 1)) == 0) {
                code = 0;
#pragma unroll
                for (int k = IMSAME_FIXED_K - 1; k >= 0; --k) code = (code << 2) | base2(seq[p - k]);
                atomicAdd(&cnt[code], 1u);
            }
        }
        codes[p] = code;
    }
}

// Entry = {x, record}: 8 bytes whatever the database size.  The reference's
// pos (last base + 1, IMSAME.c:247) is x itself below 2^32 bases (abs: the
// scan loads a hit's bases without waiting for its record's start,
// seed_kernel.hip:ent_pos), else start[record] + x (records stay < 2^32 bases).
__global__ void kmer_scatter(const uint32_t *codes, uint64_t L, const uint64_t *off, uint32_t *fill,
                             const uint64_t *st, uint64_t n_db, uint2 *ent, bool abs) {
    GRID_STRIDE(p, L) {
        const uint32_t c = codes[p];
        if (c == 0xFFFFFFFFu) continue;
        uint64_t lo = 0, hi = n_db;             // last record with start <= p
        while (hi - lo > 1) { uint64_t m = (lo + hi) >> 1; if (st[m] <= p) lo = m; else hi = m; }
        const uint64_t slot = off[c] + atomicAdd(&fill[c], 1u);
        ent[slot] = make_uint2((uint32_t)(p + 1 - (abs ? 0 : st[lo])), (uint32_t)lo);
    }
}
// the absolute entry form where positions fit (IMSAME_ENT_REL=1: the relative
// form everywhere, tests)
static bool ent_abs_for(uint64_t db_len) {
    const char *e = getenv("IMSAME_ENT_REL");
    return !(e && atoi(e)) && db_len < 0xFFFFFFFFull;
}

// records are contiguous and ascending, so descending pos = descending (record, x)
__device__ __forceinline__ uint64_t ent_key(uint2 v) { return ((uint64_t)v.y << 32) | v.x; }

// buckets in DESCENDING pos = the reference's LIFO chain order (IMSAME.c:255-276)
__global__ void segsort_small(const uint64_t *off, uint2 *ent, uint32_t *big, uint32_t *nbig) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= NBUCKETS) return;
    const uint64_t lo = off[b], n = off[b + 1] - lo;
    if (n < 2) return;
    if (n > 32) { big[atomicAdd(nbig, 1u)] = b; return; }
    uint2 *e = ent + lo;
    for (uint32_t i = 1; i < n; ++i) {
        uint2 v = e[i];
        uint32_t j = i;
        while (j > 0 && ent_key(e[j - 1]) < ent_key(v)) { e[j] = e[j - 1]; --j; }
        e[j] = v;
    }
}

// one block per large bucket (n > 32): bitonic sort, descending pos, in LDS
// when the padded bucket fits, else in a padded global scratch area.
__device__ void bitonic_desc(uint2 *s, uint32_t np) {
    for (uint32_t k = 2; k <= np; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const bool desc = (i & k) == 0;
                    if ((ent_key(s[i]) < ent_key(s[l])) == desc) { uint2 t = s[i]; s[i] = s[l]; s[l] = t; }
                }
            }
            __syncthreads();
        }
}

// block-stride over the listed buckets: past ~1 Gbase nearly every bucket
// is listed, and hbig blocks x 256 would overflow a dispatch's 2^32 items
__global__ void segsort_big(const uint64_t *off, uint2 *ent, const uint32_t *big, uint32_t nbig) {
    __shared__ uint2 s[4096];
    for (uint32_t k = blockIdx.x; k < nbig; k += gridDim.x) {
        const uint32_t b = big[k];
        const uint64_t lo = off[b], n = off[b + 1] - lo;
        uint32_t np = 1;
        while (np < n) np <<= 1;
        if (np > 4096) continue;                // handled by segsort_huge (uniform per block)
        uint2 *e = ent + lo;
        for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) s[i] = i < n ? e[i] : make_uint2(0u, 0u);
        __syncthreads();
        bitonic_desc(s, np);
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) e[i] = s[i];
        __syncthreads();                        // s is reused by the next bucket
    }
}

__global__ void segsort_huge(uint2 *e, uint32_t n, uint2 *scratch, uint32_t np) {
    for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) scratch[i] = i < n ? e[i] : make_uint2(0u, 0u);
    __syncthreads();
    bitonic_desc(scratch, np);                  // __syncthreads orders global accesses of the block
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) e[i] = scratch[i];
}

// exclusive scan of n values (1024 elements per block; recursive over block sums)
template <class TI, class TO>
__global__ void scan_blocks(const TI *in, TO *out, TO *bsum, uint64_t n) {
    __shared__ TO s[1024];
    const uint64_t i = blockIdx.x * 1024ull + threadIdx.x;
    const TO v = i < n ? (TO)in[i] : (TO)0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const TO t = threadIdx.x >= (uint32_t)o ? s[threadIdx.x - o] : (TO)0;
        __syncthreads();
        s[threadIdx.x] += t;
        __syncthreads();
    }
    if (i < n) out[i] = s[threadIdx.x] - v;
    if (threadIdx.x == 1023) bsum[blockIdx.x] = s[1023];
}
template <class T>
__global__ void scan_add(T *out, const T *bpre, uint64_t n) {
    const uint64_t i = blockIdx.x * 1024ull + threadIdx.x;
    if (i < n) out[i] += bpre[blockIdx.x];
}

// ---------------------------------------------------------------------------
// Launch order of a packed NW queue: candidates by the predicted first row of
// their read (SeedLaunch::crow) in 8-row buckets, unpredicted ones FIRST (their waves run the second
// sweep: the costliest go early, the cheap ones fill the launch's tail), so
// the candidates a wave takes share one traceback window (nw16_kernel.hip).
// Counting sort: histogram, one-block exclusive scan, scatter.
__device__ __forceinline__ uint32_t row_bucket(int32_t r, uint32_t nb) {
    if (r == INT32_MIN) return 0;
    const int64_t b = (((int64_t)r + 256) >> 3) + 1;
    return (uint32_t)(b < 1 ? 1 : b > (int64_t)nb - 1 ? (int64_t)nb - 1 : b);
}
// (grid-stride over few blocks, ROW_BLOCKS: a launch queued while other
// lanes' NW waves hold the chip waits for a slot per wave it has, as
// update_kernel)
#define ROW_BLOCKS 128u
__global__ void row_hist_kernel(const int32_t *row, uint32_t n, uint32_t nb, uint32_t *hist) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        atomicAdd(&hist[row_bucket(row[i], nb)], 1u);
}
__global__ __launch_bounds__(1024) void row_scan_kernel(const uint32_t *hist, uint32_t nb, uint32_t *cur) {
    __shared__ uint32_t sm[1024];
    const uint32_t t = threadIdx.x, per = (nb + 1023) / 1024, a = t * per;
    uint32_t sum = 0;
    for (uint32_t k = 0; k < per; ++k) if (a + k < nb) sum += hist[a + k];
    sm[t] = sum;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
        const uint32_t v = t >= o ? sm[t - o] : 0u;
        __syncthreads();
        sm[t] += v;
        __syncthreads();
    }
    uint32_t run = sm[t] - sum;
    for (uint32_t k = 0; k < per; ++k) if (a + k < nb) { cur[a + k] = run; run += hist[a + k]; }
}
__global__ void row_scatter_kernel(const int32_t *row, uint32_t n, uint32_t nb, uint32_t *cur, uint32_t *perm) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        perm[atomicAdd(&cur[row_bucket(row[i], nb)], 1u)] = i;
}

// ---------------------------------------------------------------------------
// reverse complement (replaces reverseComplement.c:21-118)
// ---------------------------------------------------------------------------
#include "revcomp_kernel.hip"

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// IMSAME_DEBUG_POISON=1: every reused device arena is filled with POISON_BYTE
// on the stream of the call that uses it -- the index build's buffers before
// the build, every per-call scratch arena at the start of each alignment call,
// the traceback / checkpoint / seam slots before each NW launch -- so a kernel
// that reads memory it did not write this call (the class of round 1's stale
// seam buffer) reads garbage instead of a plausible leftover.
// (Never at allocation: a null-stream memset is not ordered with the
// non-blocking streams that fill the buffer next.)  Debug only: results never
// depend on it.
#define POISON_BYTE 0xA5
static bool poison_on() {
    static std::once_flag f;
    static bool on = false;
    std::call_once(f, [] { const char *e = getenv("IMSAME_DEBUG_POISON"); on = e && atoi(e); });
    return on;
}

// With the flag, the host also waits for every kernel and names it on stderr
// first, so a kernel that faults on poison is the last one named.
static int poison_sync(hipStream_t s, const char *what, const void *who) {
    if (!poison_on()) return 0;
    fprintf(stderr, "[poison] %s ctx=%p\n", what, who);
    fflush(stderr);
    const hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        fprintf(stderr, "[poison] %s failed: %s\n", what, hipGetErrorString(e));
        return IMSAME_E_HIP;
    }
    return 0;
}
#define POISON_SYNC(s, what, who) do { if (int prc_ = poison_sync((s), (what), (who))) return prc_; } while (0)

struct DBuf {
    void *p = nullptr; size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr; cap = 0;
        size_t want = n + std::min<size_t>(n / 8, (size_t)1 << 30) + 4096;   // slack for regrowth, <= 1 GB
        if (hipMalloc(&p, want) != hipSuccess) { p = nullptr; return IMSAME_E_OOM; }
        cap = want;
        return 0;
    }
    int poison(hipStream_t s) const {
        return p && poison_on() && hipMemsetAsync(p, POISON_BYTE, cap, s) != hipSuccess ? IMSAME_E_HIP : 0;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
    template <class T> T *as() const { return (T *)p; }
};

struct imsame_ctx {
    int device = 0, ncu = 0;
    hipStream_t stream = nullptr;
    hipStream_t ustream = nullptr;    // query uploads (imsame_dev_set_query_range_async)
    bool ustream_own = false;         // ... a stream of its own, or the last lane's
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // round 1b (align_one): a second stream and event pair, created on first use
    hipStream_t stream_b = nullptr;
    // ... the same at the device's highest stream priority, for calls whose
    // second pipeline (weak reads' rounds) carried more NW than the first in
    // this lane's previous call (b_prio; align_one swaps it in as stream_b)
    hipStream_t stream_bh = nullptr;
    bool b_prio = false;
    hipEvent_t evb0 = nullptr, evb1 = nullptr;
    // wait events (IMSAME_WAIT block / yield, lane_sync): [0] a stream's
    // queued work, [1] the end of an NW launch; per queue (stream, stream_b)
    hipEvent_t evw[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
    // database + index; dbw: the bases 2-bit packed (seed_kernel.hip:pk_word)
    DBuf db, db_start, off, ent, brk, codes, fill, big, dbw;
    uint64_t n_db = 0, db_len = 0, n_ent = 0;
    bool ent_abs = false;             // index entries in the absolute form (kmer_scatter)
    uint32_t max_rec = 0;
    std::vector<uint64_t> h_db_start;
    bool have_index = false;
    // query: reads [q_lo, q_hi) of a query of n_q reads / q_len bases are in
    // HBM (imsame_dev_set_query_range); q holds bases [q_base, ...), q_start
    // the starts of reads q_lo .. q_hi.  Kernels index both with GLOBAL read
    // and base numbers through the biased views dev_q / dev_qs.
    DBuf q, q_start;
    DBuf qw;                          // the uploaded bases 2-bit packed, words [qw_base, qw_end) (each
    uint64_t qw_base = 0, qw_end = 0; // lane packs the words its reads use, align_one)
    uint64_t qb_end = 0;              // end of the uploaded bytes (the 64 zero bytes included)
    uint64_t n_q = 0, q_len = 0, q_lo = 0, q_hi = 0, q_base = 0, q_lo_first = 0;
    uint64_t *h_q_start = nullptr;    // starts of reads q_lo .. q_hi, page-locked (the
    uint64_t h_q_cap = 0;             // H2D copy of them runs asynchronously)
    const uint64_t *hq = nullptr;     // = h_q_start, or the parent's for a lane
    std::vector<uint32_t> h_q_bmax;   // longest read of each QB_READS block from q_lo (range_ymax)
    const uint32_t *hqb = nullptr;    // = h_q_bmax.data(), or the parent's for a lane
    bool have_query = false;
    // the upload in parts (imsame_dev_set_query_range_async): part k holds the
    // bases below q_part_end[k] and is complete when q_part_ev[k] fires (the
    // starts go first, with part 0); a lane borrows its parent's events
    std::vector<hipEvent_t> q_part_ev;
    std::vector<uint64_t> q_part_end;
    bool q_len_mult = false;         // every read length is a multiple of NW16_K
    uint32_t q_len_uni = 0;          // the one read length of the uploaded range (0: lengths differ)
    // per-read state
    DBuf res, cur_p, cur_h, memo, nmemo, rstat, act0, act1, act2, act3, cbase, ccnt, perr;
    // candidates
    DBuf cread, csid, cread2, csid2, cout, cout2;
    DBuf crow, cperm, rhist;          // predicted rows of class-0 candidates, their launch order
    DBuf cperm_b, rhist_b;            // ... of round 1b's launch (it runs beside round 1's)
    // scalars (one block of u64 counters)
    DBuf ctr;
    // tables (and the inputs they were built for)
    DBuf minraw, minlen, minident;
    bool tab_valid = false;
    long double tab_min_e = 0, tab_cov = 0, tab_id = 0;
    uint64_t tab_L = 0;
    uint32_t tab_ymax = 0, tab_xmax = 0;
    // NW scratch; the path arena of the last align (device, or host for the
    // sliced form) until imsame_dev_fetch_paths
    DBuf tb, bnd, paths, ck;
    // non-persistent nw16 launches: free-slot bitmap of the arena, 8 XCD
    // partitions (nw16_kernel.hip:nw_slot_claim); xcc_ok: 1 when the XCC_ID
    // register was seen to name 8 XCDs (nw_xcc_check), 0 no, -1 not probed
    DBuf slotbits;
    int np_part_cu = -1;              // nw16_np_part_cu (-1: not computed)
    // the arena of non-persistent launches: ONE per device context, shared by
    // its lanes (np_owner) -- slots are taken per wave, so every NW launch of
    // every lane draws from the chip's residency in one arena (np_prepare)
    DBuf np_tb, np_ck;
    imsame_ctx *np_owner = nullptr;   // lanes: the context whose arena they use
    uint64_t paths_cap_dev = 0, paths_n = 0;
    double paths_hint = 0;     // path entries per read of the last call
    std::vector<uint32_t> paths_host;
    bool paths_on_host = false;
    // revcomp
    DBuf rc_in, rc_out, rc_a, rc_b, rc_c;
    // database slices (imsame_dev_align_sliced): the e-value's L_DB is the
    // whole database's length, and each read scans windows below its cap
    uint64_t ev_db_len = 0;          // 0: db_len
    bool use_wcap = false, use_wstart = false;
    DBuf wcap, wout, wstart;
    // LANES 1, 2, ...: contexts sharing this one's index and query (aliased
    // buffers), each with its own stream and per-read state, so the parts of
    // one call run concurrently (see imsame_dev_align)
    std::vector<imsame_ctx *> subs;   // lanes 1, 2, ...
    bool is_sub = false, paths_split = false;
    std::vector<uint64_t> lane_paths; // path entries of lanes 1, 2, ... after a split call
    // NW launch intervals (ms since the call's origin event) for the busy time
    hipEvent_t origin = nullptr;
    hipEvent_t ev_w = nullptr;        // align_one: round 1's unpredicted candidates updated (pipelines)
    hipEvent_t ev_wd = nullptr;       // align_one: the weak launch and its update ended (pipelines)
    std::vector<std::pair<float, float>> nw_iv;
    // IMSAME_DEBUG_TIMELINE: (kind 'S' seed / 'N' NW, round, items, start, end)
    struct TlEv { char kind; int round; uint32_t n; float a, b; };
    std::vector<TlEv> tl;
    int cur_round = 0;
    // the call's two read pipelines (align_one: pipe_rounds) append launch
    // intervals and timeline events from two host threads; a launch that is
    // not non-persistent uses this lane's own arena, one at a time
    std::mutex iv_mu, persist_mu;
    int nlanes = 1;                   // lanes of the running call (the seed scan's group size
                                      // follows the reads scanned across all of them)
    std::vector<uint32_t> part_paths; // host copy of this lane's paths for an imsame_dev_align_parts callback
};

static inline uint64_t hqs(const imsame_ctx *c, uint64_t r) { return c->hq[r - c->q_lo]; }
// longest read of [a, b) within the uploaded range: block maxima (set at
// upload) for the whole blocks, a scan of the ragged ends
#define QB_READS 4096
static uint64_t range_ymax(const imsame_ctx *c, uint64_t a, uint64_t b) {
    uint64_t m = 0;
    auto len = [&](uint64_t r) { return hqs(c, r + 1) - hqs(c, r); };
    uint64_t blk = (a - c->q_lo + QB_READS - 1) / QB_READS, r = c->q_lo + blk * QB_READS;
    for (uint64_t x = a; x < std::min(b, r); ++x) m = std::max(m, len(x));
    for (; r + QB_READS <= b; r += QB_READS, ++blk) m = std::max<uint64_t>(m, c->hqb[blk]);
    for (uint64_t x = std::max(a, r); x < b; ++x) m = std::max(m, len(x));
    return m;
}
// biased views: valid for the uploaded reads (and QPAD bases before them)
static inline const uint8_t *dev_q(const imsame_ctx *c) { return (const uint8_t *)((uintptr_t)c->q.p - c->q_base); }
static inline const uint32_t *dev_qw(const imsame_ctx *c) {
    return (const uint32_t *)((uintptr_t)c->qw.p - c->qw_base * sizeof(uint32_t));
}
static inline const uint64_t *dev_qs(const imsame_ctx *c) {
    return (const uint64_t *)((uintptr_t)c->q_start.p - c->q_lo * sizeof(uint64_t));
}
// bases uploaded before a range's first read: the borrowed base (Q4) and the
// 16-byte chunk loads of the ungapped extension reach back <= 18 bases
#define QPAD 64

// counters block layout (u64 slots)
enum { C_NCAND = 0, C_NCAND2, C_NNEXT, C_NCANDB, C_NCAND2B, C_NNEXT2, C_WORKB,   // (round 1b: B, 2)
       C_WORK, C_WORK2, C_PATHS, C_FLAGS, C_ERR, C_HITS, C_CELLS, C_NACC, C_REDO,
       C_PROF, C_WIN = C_PROF + 12, C_FBK, C_SWORK, C_DBG = C_SWORK + 3, C_WASTE = C_DBG + 8,
       C_NSLOTS };

static double now_ms() {
    struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

extern "C" void imsame_params_default(imsame_params *p) {
    memset(p, 0, sizeof *p);
    p->min_e = 1 / powl(10, 20);                         // IMSAME.c:44
    p->min_coverage = 0.5; p->min_identity = 0.5;        // :46
    p->igap = -5; p->egap = -2;                          // :47
    p->max_read_size = IMSAME_MAX_READ_SIZE;
    p->want_paths = 0;
}

extern "C" const char *imsame_strerror(int code) {
    switch (code) {
    case IMSAME_OK: return "ok";
    case IMSAME_E_HIP: return "HIP runtime error";
    case IMSAME_E_OOM: return "out of memory";
    case IMSAME_E_READ_TOO_LONG: return "Read size reached for gapped alignment.";
    case IMSAME_E_ARG: return "bad argument";
    case IMSAME_E_RANGE: return "gap parameters out of int32 range";
    case IMSAME_E_PATHS: return "path arena too small";
    case IMSAME_E_STATE: return "index or query not loaded";
    }
    return "unknown error";
}

// Hardware queues: HIP maps a process's streams onto GPU_MAX_HW_QUEUES
// hardware queues (4 when unset), and two lanes whose streams share a queue
// serialize completely (rocprofv3 trace, profiles/r2ag_lane_timeline.txt).
// The library never changes the variable (it is the host program's to set,
// before its first HIP call: the imsame CLI and bench.py ask for 8); it reads
// the value the runtime started with, once, and sizes its lanes to it.
static int hw_queues() {
    static std::once_flag f;
    static int q = 4;
    std::call_once(f, [] {
        const char *e = getenv("GPU_MAX_HW_QUEUES");
        const int v = e ? atoi(e) : 0;
        q = v > 0 ? v : 4;
    });
    return q;
}

// Most lanes a call runs (imsame_dev_align): a lane has two streams (its
// rounds and round 1b's scan + NW launch, align_one), each wants a hardware
// queue of its own -- a stream that shares one waits behind the other's
// kernels (C2 with 8 lanes on 8 queues: lane 0's round-1b launch ran 75 ms
// late, profiles/r3_c2_timeline.txt) -- so queues / 2, <= 8 (C2, 8 queues:
// 4 lanes, 119.3-119.9 vs 121.0-121.6 ms with 8, profiles/r3q16/).
#define LANES_MAX 8
#define LANES_DEF 3                 // lanes a call uses by default (align_impl); more are added on demand
static int lanes_for_queues() { return std::max(1, std::min(LANES_MAX, hw_queues() / 2)); }

// Host threads and waits.  A lane's host thread spends most of a call
// waiting for its stream (counters of a round, the end of an NW launch);
// hipStreamSynchronize / hipEventSynchronize on a plain event spin that
// thread.  A rank of an N-GPU run may have fewer CPUs than its lanes and
// upload threads (bench.py gives each rank an equal share of the host's
// usable CPUs): IMSAME_HOST_THREADS caps the threads of the upload's host
// pass and the lanes of a call (one host thread each), and IMSAME_WAIT=block
// makes the lanes wait on events created with hipEventBlockingSync (the
// thread sleeps until the device signals), IMSAME_WAIT=yield poll their event
// and yield the CPU between polls.
static int host_threads_cap() {
    static std::once_flag f;
    static int n = 8;
    std::call_once(f, [] { const char *e = getenv("IMSAME_HOST_THREADS"); if (e && atoi(e) > 0) n = std::min(8, atoi(e)); });
    return n;
}
enum { WAIT_SPIN = 0, WAIT_BLOCK, WAIT_YIELD };
static int wait_mode() {
    static std::once_flag f;
    static int m = WAIT_SPIN;
    std::call_once(f, [] {
        // yield by default: as fast as HIP's spinning sync with a CPU per
        // thread, and it keeps a rank whose CPU share is below its threads
        // from starving the runtime's own threads (C2 1/8 shard on 2 CPUs, 3
        // lanes: 17.1 vs 18.3 ms; 16 CPUs: 16.38 vs 16.46; C2 106.4 vs 106.2;
        // profiles/r5d/)
        const char *e = getenv("IMSAME_WAIT");
        m = !e ? WAIT_YIELD : !strcmp(e, "block") ? WAIT_BLOCK : !strcmp(e, "spin") ? WAIT_SPIN : WAIT_YIELD;
    });
    return m;
}
static bool wait_block() { return wait_mode() != WAIT_SPIN; }   // waits go through the evw events
// wait until event e (recorded) has completed
static int ev_wait(hipEvent_t e) {
    if (wait_mode() == WAIT_YIELD) {
        for (;;) {
            const hipError_t q = hipEventQuery(e);
            if (q == hipSuccess) return 0;
            if (q != hipErrorNotReady) return IMSAME_E_HIP;
            sched_yield();
        }
    }
    HIPCHK(hipEventSynchronize(e));
    return 0;
}
// wait for everything queued on s (s: the lane's stream or its round-1b stream)
static int lane_sync(imsame_ctx *c, hipStream_t s) {
    if (!wait_block()) { HIPCHK(hipStreamSynchronize(s)); return 0; }
    hipEvent_t e = c->evw[s == c->stream_b ? 1 : 0][0];
    HIPCHK(hipEventRecord(e, s));
    return ev_wait(e);
}
#define LANE_SYNC(c, s) do { if (int lrc_ = lane_sync((c), (s))) return lrc_; } while (0)

extern "C" int imsame_dev_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

// Non-persistent packed launches need the XCD of each wave (nw_slot_claim):
// a probe kernel reads XCC_ID in 512 blocks, which must name each of 8 XCDs.
// Off when the check fails (persistent launches then), or IMSAME_NW_PERSIST=1.
// The probe runs once per device and process, when a context is created
// (ctx_create: nothing of this process runs yet, and its hipFree -- which
// waits for the whole device -- stalls no lane).
static std::mutex g_xcc_mu;
static int g_xcc_ok[64];                   // 0 not probed, 1 ok, 2 failed
static void xcc_probe_device(imsame_ctx *c) {
    std::lock_guard<std::mutex> lk(g_xcc_mu);
    const int d = c->device & 63;
    if (g_xcc_ok[d]) return;
    g_xcc_ok[d] = 2;
    if (c->ncu % 8 || c->ncu < 64) return;
    const unsigned nb = 512;
    DBuf b;
    if (b.ensure(nb * 4)) return;
    std::vector<uint32_t> h(nb, 0xFFFFFFFFu);
    xcc_probe_kernel<<<nb, 64, 0, c->stream>>>(b.as<uint32_t>());
    bool ok = hipGetLastError() == hipSuccess &&
              hipMemcpyAsync(h.data(), b.p, nb * 4, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
              hipStreamSynchronize(c->stream) == hipSuccess;
    uint32_t seen = 0;
    for (uint32_t v : h) { if (v >= 8) ok = false; else seen |= 1u << v; }
    b.release();
    g_xcc_ok[d] = ok && seen == 0xFFu ? 1 : 2;
}
static bool nw_xcc_check(imsame_ctx *c) {
    const char *pe = getenv("IMSAME_NW_PERSIST");
    if (pe && atoi(pe)) return false;
    std::lock_guard<std::mutex> lk(g_xcc_mu);
    return g_xcc_ok[c->device & 63] == 1;
}

// A context with its compute stream (imsame_dev_open adds the upload stream).
static int ctx_create(int device, imsame_ctx **out) {
    HIPCHK(hipSetDevice(device));
    imsame_ctx *c = new imsame_ctx();
    c->device = device;
    // CU count: one attribute query (hipGetDeviceProperties fills the whole
    // struct and costs milliseconds per context)
    HIPCHK(hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, device));
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreate(&c->ev0));
    HIPCHK(hipEventCreate(&c->ev1));
    for (int k = 0; k < 2; ++k)
        HIPCHK(hipEventCreateWithFlags(&c->evw[0][k], hipEventBlockingSync | hipEventDisableTiming));
    if (c->ctr.ensure(C_NSLOTS * 8)) { delete c; return IMSAME_E_OOM; }
    xcc_probe_device(c);
    *out = c;
    return IMSAME_OK;
}

static int lane_add(imsame_ctx *c) {
    imsame_ctx *l = nullptr;
    const int rc = ctx_create(c->device, &l);
    if (rc) return rc;
    l->is_sub = true;
    c->subs.push_back(l);
    return 0;
}

extern "C" int imsame_dev_open(int device, imsame_ctx **out) {
    const bool dbg = getenv("IMSAME_DEBUG_OPEN") != nullptr;   // diagnostics: where the open's time goes
    const double t0 = dbg ? now_ms() : 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return IMSAME_E_HIP;
    const double t1 = dbg ? now_ms() : 0;
    imsame_ctx *c = nullptr;
    int rc = ctx_create(device, &c);
    if (rc) return rc;
    const double t2 = dbg ? now_ms() : 0;
    // Stream creation order fixes the hardware queues: the runtime gives each
    // new stream a queue of its own until GPU_MAX_HW_QUEUES are in use, then
    // shares the least used one.  So the compute streams of this context and
    // its lanes come first, one queue each, and the upload stream last, on the
    // last lane's queue (that lane starts after the whole upload anyway).
    const int nl = std::min(lanes_for_queues(), LANES_DEF);
    for (int k = 1; k < nl && !rc; ++k) rc = lane_add(c);
    const double t3 = dbg ? now_ms() : 0;
    // the query upload runs on the last lane's compute stream (that lane's
    // rounds wait for the upload's last part anyway): each stream with a
    // hardware queue of its own costs ~19 ms of the open (IMSAME_DEBUG_OPEN,
    // profiles/r4r/; creating them on parallel threads gains nothing, the
    // runtime serialises it); a context without lanes has a stream of its own
    // for it, so its rounds overlap the upload
    if (!rc && !c->subs.empty()) c->ustream = c->subs.back()->stream;
    else if (!rc && hipStreamCreateWithFlags(&c->ustream, hipStreamNonBlocking) == hipSuccess) c->ustream_own = true;
    else if (!rc) rc = IMSAME_E_HIP;
    // round 1b's streams (align_one) after the lanes' compute streams: they
    // share the hardware queues the runtime has left (created here, not in a
    // call: creating one while other lanes run stalled a CLI call for 4.8 s,
    // profiles/r3r_*)
    int prio_lo = 0, prio_hi = 0;
    if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) rc = IMSAME_E_HIP;
    const char *pbe = getenv("IMSAME_PRIO_B");
    const bool no_bh = pbe && !atoi(pbe);         // (prio_b off: no high-priority streams at all)
    for (size_t k = 0; k <= c->subs.size() && !rc; ++k) {
        imsame_ctx *l = k ? c->subs[k - 1] : c;
        if (hipStreamCreateWithFlags(&l->stream_b, hipStreamNonBlocking) != hipSuccess ||
            (!no_bh && hipStreamCreateWithPriority(&l->stream_bh, hipStreamNonBlocking, prio_hi) != hipSuccess) ||
            hipEventCreate(&l->evb0) != hipSuccess || hipEventCreate(&l->evb1) != hipSuccess ||
            hipEventCreateWithFlags(&l->evw[1][0], hipEventBlockingSync | hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&l->evw[1][1], hipEventBlockingSync | hipEventDisableTiming) != hipSuccess)
            rc = IMSAME_E_HIP;
    }
    if (rc) { imsame_dev_close(c); return rc; }
    if (dbg)
        fprintf(stderr, "[imsame] open_ms {\"runtime\": %.2f, \"context\": %.2f, \"lanes\": %.2f, \"streams\": %.2f}\n",
                t1 - t0, t2 - t1, t3 - t2, now_ms() - t3);
    *out = c;
    return IMSAME_OK;
}

static void lane_unalias(imsame_ctx *l) {
    DBuf *al[] = {&l->db, &l->db_start, &l->off, &l->ent, &l->q, &l->q_start, &l->dbw, &l->qw};
    for (DBuf *b : al) { b->p = nullptr; b->cap = 0; }
    l->q_part_ev.clear(); l->q_part_end.clear();
}

extern "C" void imsame_dev_close(imsame_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->ustream) (void)hipStreamSynchronize(c->ustream);    // before the lane that may own it goes
    if (!c->ustream_own) c->ustream = nullptr;
    for (imsame_ctx *l : c->subs) { lane_unalias(l); imsame_dev_close(l); }
    c->subs.clear();
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    DBuf *bufs[] = {&c->db, &c->db_start, &c->off, &c->ent, &c->brk, &c->codes, &c->fill, &c->big, &c->q,
                    &c->q_start, &c->res, &c->cur_p, &c->cur_h, &c->memo, &c->nmemo, &c->rstat, &c->act0,
                    &c->act1, &c->cread, &c->csid, &c->cread2, &c->csid2, &c->cout, &c->cout2, &c->ctr,
                    &c->minraw, &c->minlen, &c->minident, &c->tb, &c->bnd, &c->paths, &c->ck, &c->rc_in, &c->rc_out,
                    &c->rc_a, &c->rc_b, &c->rc_c, &c->cbase, &c->ccnt, &c->perr, &c->wcap, &c->wout, &c->wstart,
                    &c->crow, &c->cperm, &c->rhist, &c->act2, &c->act3, &c->slotbits, &c->np_tb, &c->np_ck, &c->dbw, &c->qw,
                    &c->cperm_b, &c->rhist_b};
    for (DBuf *b : bufs) b->release();
    (void)hipEventDestroy(c->ev0);
    (void)hipEventDestroy(c->ev1);
    if (c->evb0) (void)hipEventDestroy(c->evb0);
    if (c->ev_w) (void)hipEventDestroy(c->ev_w);
    if (c->ev_wd) (void)hipEventDestroy(c->ev_wd);
    if (c->evb1) (void)hipEventDestroy(c->evb1);
    for (auto &q : c->evw)
        for (hipEvent_t e : q) if (e) (void)hipEventDestroy(e);
    if (c->stream_b) (void)hipStreamDestroy(c->stream_b);
    if (c->stream_bh) (void)hipStreamDestroy(c->stream_bh);
    if (c->origin && !c->is_sub) (void)hipEventDestroy(c->origin);     // a lane borrows its parent's
    if (!c->is_sub)
        for (hipEvent_t e : c->q_part_ev) (void)hipEventDestroy(e);
    if (!c->is_sub && c->h_q_start) (void)hipHostFree(c->h_q_start);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->ustream && c->ustream_own) (void)hipStreamDestroy(c->ustream);
    delete c;
}

// Lane k >= 1 of c, aliasing c's index and query (not owned).  Lanes beyond
// the hardware queues (IMSAME_LANES) are added on demand and share queues.
static int lane_sub(imsame_ctx *c, int k, imsame_ctx **out) {
    while ((int)c->subs.size() < k) {
        const int rc = lane_add(c);
        if (rc) return rc;
    }
    imsame_ctx *l = c->subs[k - 1];
    l->db = c->db; l->db_start = c->db_start; l->off = c->off; l->ent = c->ent; l->q = c->q; l->q_start = c->q_start;
    l->dbw = c->dbw; l->qw = c->qw; l->qw_base = c->qw_base; l->qw_end = c->qw_end; l->qb_end = c->qb_end;
    l->n_db = c->n_db; l->db_len = c->db_len; l->n_ent = c->n_ent; l->max_rec = c->max_rec; l->ent_abs = c->ent_abs;
    l->have_index = c->have_index;
    l->n_q = c->n_q; l->q_len = c->q_len; l->q_lo = c->q_lo; l->q_hi = c->q_hi; l->q_base = c->q_base;
    l->q_lo_first = c->q_lo_first; l->hq = c->hq; l->hqb = c->hqb; l->have_query = c->have_query;
    l->q_len_mult = c->q_len_mult; l->q_len_uni = c->q_len_uni;
    l->q_part_ev = c->q_part_ev; l->q_part_end = c->q_part_end;
    l->ev_db_len = 0; l->use_wcap = l->use_wstart = false;
    l->np_owner = c;
    *out = l;
    return 0;
}

static unsigned nblk(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

// grid for a grid-stride kernel (a dispatch holds < 2^32 work-items)
static unsigned gsblk(uint64_t n, unsigned b) { return (unsigned)std::min<uint64_t>((n + b - 1) / b, 1u << 20); }

// exclusive scan out[0..n) of in[0..n) (TO wraps past its range: callers size for it)
template <class TI, class TO>
static int dev_scan(hipStream_t s, const TI *in, TO *out, uint64_t n) {
    if (n == 0) return 0;
    const uint64_t nb = (n + 1023) / 1024;
    DBuf bs, bp;
    if (bs.ensure(nb * sizeof(TO) + 16) || bp.ensure(nb * sizeof(TO) + 16)) return IMSAME_E_OOM;
    scan_blocks<TI, TO><<<(unsigned)nb, 1024, 0, s>>>(in, out, bs.as<TO>(), n);
    if (nb > 1) {
        int rc = dev_scan<TO, TO>(s, bs.as<TO>(), bp.as<TO>(), nb);
        if (rc) return rc;
        scan_add<TO><<<(unsigned)nb, 1024, 0, s>>>(out, bp.as<TO>(), n);
    }
    HIPCHK(hipStreamSynchronize(s));     // the level buffers are freed on return
    return 0;
}

extern "C" int imsame_dev_index(imsame_ctx *c, const uint8_t *db_seq, uint64_t db_len, const uint64_t *db_start,
                                uint64_t n_db, const uint8_t *db_brk) {
    if (!c || (db_len && !db_seq) || (n_db && !db_start)) return IMSAME_E_ARG;
    if (n_db >= 0xFFFFFFF0ull) return IMSAME_E_ARG;              // u32 record ids
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    c->have_index = false;
    c->n_db = n_db; c->db_len = db_len;
    c->h_db_start.assign(db_start, db_start + n_db);
    c->h_db_start.push_back(db_len);
    c->max_rec = 0;
    uint64_t max_rec = 0;
    for (uint64_t k = 0; k < n_db; ++k) max_rec = std::max<uint64_t>(max_rec, c->h_db_start[k + 1] - c->h_db_start[k]);
    if (max_rec >= 0xFFFFFFF0ull) return IMSAME_E_ARG;           // record-relative u32 entry positions
    c->max_rec = (uint32_t)max_rec;
    const uint64_t nw = db_len / 32 + 2, npw = db_len / 16 + 4;
    if (c->db.ensure(db_len + 64) || c->dbw.ensure(npw * 4) || c->db_start.ensure((n_db + 1) * 8) || c->brk.ensure(nw * 4) ||
        c->codes.ensure((db_len + 1) * 4) || c->off.ensure(((uint64_t)NBUCKETS + 1) * 8) ||
        c->fill.ensure((uint64_t)NBUCKETS * 4) || c->big.ensure((uint64_t)NBUCKETS * 4))
        return IMSAME_E_OOM;
    {
        const DBuf *scr[] = {&c->db, &c->codes, &c->off, &c->fill, &c->big, &c->ent};
        for (const DBuf *b : scr)
            if (int rc = b->poison(s)) return rc;
    }
    if (db_len) HIPCHK(hipMemcpyAsync(c->db.p, db_seq, db_len, hipMemcpyHostToDevice, s));
    uint64_t *badf = c->ctr.as<uint64_t>() + C_FLAGS;  // bit 3: a byte that is not ACGT (no align runs now)
    HIPCHK(hipMemsetAsync(badf, 0, 8, s));
    pack2_kernel<<<gsblk(npw, 256), 256, 0, s>>>(c->db.as<uint8_t>(), 0, (int64_t)db_len, c->dbw.as<uint32_t>(), 0, npw,
                                                 (unsigned long long *)badf);
    HIPCHK(hipMemcpyAsync(c->db_start.p, c->h_db_start.data(), (n_db + 1) * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(c->brk.p, 0, nw * 4, s));
    if (db_brk && db_len) HIPCHK(hipMemcpyAsync(c->brk.p, db_brk, (db_len + 7) / 8, hipMemcpyHostToDevice, s));
    if (n_db) mark_record_starts<<<nblk(n_db, 256), 256, 0, s>>>(c->db_start.as<uint64_t>(), n_db, db_len,
                                                                   c->brk.as<uint32_t>());
    HIPCHK(hipMemsetAsync(c->fill.p, 0, (uint64_t)NBUCKETS * 4, s));
    if (db_len) kmer_code_kernel<<<gsblk(db_len, 256), 256, 0, s>>>(c->db.as<uint8_t>(), db_len, c->brk.as<uint32_t>(),
                                                                  c->codes.as<uint32_t>(), c->fill.as<uint32_t>());
    POISON_SYNC(s, "kmer_code_kernel", c);
    // exclusive scan of the counts -> off[0..NB], off[NB] = total
    uint64_t total = 0;
    {
        DBuf cnt;
        if (cnt.ensure(((uint64_t)NBUCKETS + 1) * 4)) return IMSAME_E_OOM;
        HIPCHK(hipMemsetAsync(cnt.p, 0, ((uint64_t)NBUCKETS + 1) * 4, s));
        HIPCHK(hipMemcpyAsync(cnt.p, c->fill.p, (uint64_t)NBUCKETS * 4, hipMemcpyDeviceToDevice, s));
        int rc = dev_scan<uint32_t, uint64_t>(s, cnt.as<uint32_t>(), c->off.as<uint64_t>(), (uint64_t)NBUCKETS + 1);
        if (rc) return rc;
        HIPCHK(hipMemcpyAsync(&total, c->off.as<uint64_t>() + NBUCKETS, 8, hipMemcpyDeviceToHost, s));
        uint64_t hbad = 0;
        HIPCHK(hipMemcpyAsync(&hbad, badf, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        cnt.release();
        if (hbad) return IMSAME_E_ARG;                 // not an ACGT-filtered database (the header)
    }
    c->n_ent = total;
    c->ent_abs = ent_abs_for(db_len);
    if (c->ent.ensure((total + 1) * 8)) return IMSAME_E_OOM;
    HIPCHK(hipMemsetAsync(c->fill.p, 0, (uint64_t)NBUCKETS * 4, s));
    if (db_len) kmer_scatter<<<gsblk(db_len, 256), 256, 0, s>>>(c->codes.as<uint32_t>(), db_len, c->off.as<uint64_t>(),
                                                              c->fill.as<uint32_t>(), c->db_start.as<uint64_t>(), n_db,
                                                              c->ent.as<uint2>(), c->ent_abs);
    POISON_SYNC(s, "kmer_scatter", c);
    uint32_t *nbig = c->fill.as<uint32_t>();       // fill is free again: reuse as a counter
    HIPCHK(hipMemsetAsync(nbig, 0, 4, s));
    segsort_small<<<nblk(NBUCKETS, 256), 256, 0, s>>>(c->off.as<uint64_t>(), c->ent.as<uint2>(),
                                                      c->big.as<uint32_t>(), nbig);
    POISON_SYNC(s, "segsort_small", c);
    uint32_t hbig = 0;
    HIPCHK(hipMemcpyAsync(&hbig, nbig, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (hbig) {
        segsort_big<<<std::min<uint32_t>(hbig, 1u << 16), 256, 0, s>>>(c->off.as<uint64_t>(), c->ent.as<uint2>(),
                                                                      c->big.as<uint32_t>(), hbig);
        // buckets beyond 4096 entries (repeats): one block each, padded global scratch
        std::vector<uint32_t> bigs(hbig);
        std::vector<uint64_t> offs(NBUCKETS + 1);
        HIPCHK(hipMemcpyAsync(bigs.data(), c->big.p, (uint64_t)hbig * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(offs.data(), c->off.p, ((uint64_t)NBUCKETS + 1) * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        DBuf scr;
        for (uint32_t b : bigs) {
            const uint32_t nb = (uint32_t)(offs[b + 1] - offs[b]);
            uint32_t np = 1;
            while (np < nb) np <<= 1;
            if (np <= 4096) continue;
            if (scr.ensure((uint64_t)np * 8)) return IMSAME_E_OOM;
            segsort_huge<<<1, 1024, 0, s>>>(c->ent.as<uint2>() + offs[b], nb, scr.as<uint2>(), np);
        }
        HIPCHK(hipStreamSynchronize(s));
        scr.release();
    }
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipGetLastError());
    c->codes.release();
    c->have_index = true;
    return IMSAME_OK;
}

// parts of an asynchronous query upload (each a few tens of MB at C2)
#define Q_PARTS 8

extern "C" int imsame_dev_set_query_range_async(imsame_ctx *c, const uint8_t *q_seq, uint64_t q_len,
                                                const uint64_t *q_start, uint64_t n_q, uint64_t read_from,
                                                uint64_t read_to) {
    if (!c || c->is_sub || (q_len && !q_seq) || (n_q && !q_start) || read_from > read_to || read_to > n_q)
        return IMSAME_E_ARG;
    if (n_q >= 0xFFFFFFF0ull) return IMSAME_E_ARG;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->ustream));    // a previous upload may still read h_q_start / fill q
    c->have_query = false;
    auto qs = [&](uint64_t r) { return r < n_q ? q_start[r] : q_len; };
    // one pass over the shard's starts: ascending within the query (else
    // IMSAME_E_ARG), the host copy, every length a multiple of NW16_K?, and
    // the longest read of each QB_READS block (range_ymax)
    const uint64_t m = read_to - read_from;
    if (c->h_q_cap < m + 1) {
        if (c->h_q_start) HIPCHK(hipHostFree(c->h_q_start));
        c->h_q_start = nullptr; c->h_q_cap = 0;
        const uint64_t cap = (m + 1) + (m + 1) / 8 + 1024;
        if (hipHostMalloc((void **)&c->h_q_start, cap * 8, hipHostMallocDefault) != hipSuccess) {
            c->h_q_start = nullptr;
            return IMSAME_E_OOM;
        }
        c->h_q_cap = cap;
    }
    c->h_q_bmax.assign(m / QB_READS + 1, 0);
    uint64_t *h = c->h_q_start;
    uint32_t *bm = c->h_q_bmax.data();
    h[0] = qs(read_from);
    // reads k-1 (k = 1 .. m) in chunks of whole blocks, one host thread each
    // (1M reads: ~1 ms on one core, on the critical path of every upload)
    auto pass = [&](uint64_t k0, uint64_t k1, bool *okp, bool *multp, uint64_t *lminp) {
        uint64_t prev = k0 == 1 ? h[0] : qs(read_from + k0 - 1);
        bool ok = true, mult = true;
        uint64_t lmin = ~0ull;
        for (uint64_t k = k0; k < k1; ++k) {
            const uint64_t v = read_from + k < n_q ? q_start[read_from + k] : q_len;
            const uint64_t len = v - prev;
            ok &= v >= prev;
            mult &= len % NW16_K == 0;
            lmin = std::min(lmin, len);
            uint32_t &b = bm[(k - 1) / QB_READS];
            b = std::max<uint32_t>(b, (uint32_t)std::min<uint64_t>(len, 0xFFFFFFFFu));
            h[k] = v;
            prev = v;
        }
        *okp = ok; *multp = mult; *lminp = lmin;
    };
    const uint64_t nblk_r = (m + QB_READS - 1) / QB_READS;
    const int nt = (int)std::min<uint64_t>(host_threads_cap(), (nblk_r + 15) / 16);   // >= 16 blocks per thread
    bool okv[8] = {true, true, true, true, true, true, true, true}, mv[8] = {true, true, true, true, true, true, true, true};
    uint64_t lminv[8] = {~0ull, ~0ull, ~0ull, ~0ull, ~0ull, ~0ull, ~0ull, ~0ull};
    if (nt <= 1) {
        pass(1, m + 1, &okv[0], &mv[0], &lminv[0]);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) {
            const uint64_t k0 = 1 + (nblk_r * t / nt) * QB_READS, k1 = std::min<uint64_t>(1 + (nblk_r * (t + 1) / nt) * QB_READS, m + 1);
            th.emplace_back(pass, k0, k1, &okv[t], &mv[t], &lminv[t]);
        }
        for (auto &x : th) x.join();
    }
    bool ok = h[0] <= q_len, mult = true;
    uint64_t lmin = ~0ull, lmax = 0;
    for (int t = 0; t < 8; ++t) { ok = ok && okv[t]; mult = mult && mv[t]; lmin = std::min(lmin, lminv[t]); }
    for (uint32_t b : c->h_q_bmax) lmax = std::max<uint64_t>(lmax, b);
    const uint64_t prev = h[m];
    if (!ok || prev > q_len) return IMSAME_E_ARG;                   // starts ascend within the query
    c->n_q = n_q; c->q_len = q_len; c->q_lo = read_from; c->q_hi = read_to;
    c->hq = c->h_q_start;
    c->hqb = c->h_q_bmax.data();
    // reads q_lo_first .. read_from-1 are empty (start where read_from starts)
    uint64_t f = read_from;
    while (f > 0 && qs(f - 1) == qs(read_from)) --f;
    c->q_lo_first = f;
    const uint64_t b0 = qs(read_from), b1 = qs(read_to);
    c->q_base = b0 > QPAD ? b0 - QPAD : 0;
    const uint64_t nb = b1 - c->q_base, ns = read_to - read_from + 1;
    c->q_len_mult = mult;
    c->q_len_uni = (m > 0 && lmin == lmax && lmax < 0xFFFFFFFFu) ? (uint32_t)lmax : 0u;
    // packed copy: words qw_base .. qw_end of the bases [q_base, q_base + nb + 64)
    c->qw_base = c->q_base >> 4;
    const uint64_t qw_end = (c->q_base + nb + 64) / 16 + 2;
    if (c->q.ensure(nb + 64) || c->q_start.ensure(ns * 8) || c->qw.ensure((qw_end - c->qw_base) * 4))
        return IMSAME_E_OOM;
    while (c->q_part_ev.size() < Q_PARTS) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->q_part_ev.push_back(e);
    }
    c->q_part_end.assign(Q_PARTS, 0);
    // on the upload stream: every lane (this context's stream included) waits
    // only for the parts that hold its reads
    HIPCHK(hipMemcpyAsync(c->q_start.p, c->h_q_start, ns * 8, hipMemcpyHostToDevice, c->ustream));
    HIPCHK(hipMemsetAsync((uint8_t *)c->q.p + nb, 0, 64, c->ustream));
    // (the packed copy the seed scan reads, qw, is made by each lane over its
    // own reads once their parts are in HBM: align_one)
    c->qw_end = qw_end; c->qb_end = c->q_base + nb + 64;
    for (uint64_t k = 0, a = 0; k < Q_PARTS; ++k) {      // bases [q_base + a, q_base + b)
        const uint64_t b = nb * (k + 1) / Q_PARTS;
        if (b > a) HIPCHK(hipMemcpyAsync((uint8_t *)c->q.p + a, q_seq + c->q_base + a, b - a, hipMemcpyHostToDevice,
                                         c->ustream));
        HIPCHK(hipEventRecord(c->q_part_ev[k], c->ustream));
        c->q_part_end[k] = c->q_base + b;
        a = b;
    }
    c->have_query = true;
    POISON_SYNC(c->ustream, "query upload", c);
    return IMSAME_OK;
}

// stream s waits until the uploaded bases below `end` are in HBM
static int query_wait(imsame_ctx *c, hipStream_t s, uint64_t end) {
    for (size_t k = 0; k < c->q_part_end.size(); ++k)
        if (k + 1 == c->q_part_end.size() || c->q_part_end[k] >= end) {
            HIPCHK(hipStreamWaitEvent(s, c->q_part_ev[k], 0));
            break;
        }
    return 0;
}

extern "C" int imsame_dev_sync(imsame_ctx *c) {
    if (!c) return IMSAME_E_ARG;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->ustream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return IMSAME_OK;
}

extern "C" int imsame_dev_set_query_range(imsame_ctx *c, const uint8_t *q_seq, uint64_t q_len,
                                          const uint64_t *q_start, uint64_t n_q, uint64_t read_from,
                                          uint64_t read_to) {
    const int rc = imsame_dev_set_query_range_async(c, q_seq, q_len, q_start, n_q, read_from, read_to);
    return rc ? rc : imsame_dev_sync(c);
}

extern "C" int imsame_dev_set_query(imsame_ctx *c, const uint8_t *q_seq, uint64_t q_len, const uint64_t *q_start,
                                    uint64_t n_q) {
    return imsame_dev_set_query_range(c, q_seq, q_len, q_start, n_q, 0, n_q);
}

extern "C" void *imsame_host_alloc(uint64_t bytes) {
    void *p = nullptr;
    return hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) == hipSuccess ? p : nullptr;
}

extern "C" void imsame_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

static int build_tables(imsame_ctx *c, const imsame_params *p, uint32_t ymax, uint32_t xmax) {
    // the tables depend on the thresholds, L_DB and the shape only: reuse
    // them across calls (ymax = 10,000 takes ~0.1 s of x87 expl / divisions)
    const uint64_t L = c->ev_db_len ? c->ev_db_len : c->db_len;
    if (c->tab_valid && c->tab_min_e == p->min_e && c->tab_cov == p->min_coverage && c->tab_id == p->min_identity &&
        c->tab_L == L && c->tab_ymax == ymax && c->tab_xmax == xmax)
        return 0;
    c->tab_valid = false;
    std::vector<uint64_t> mr;
    std::vector<uint32_t> ml, mi;
    imsame_build_tables(p, c->ev_db_len ? c->ev_db_len : c->db_len, ymax, xmax, mr, ml, mi);
    if (c->minraw.ensure(mr.size() * 8) || c->minlen.ensure(ml.size() * 4) || c->minident.ensure(mi.size() * 4))
        return IMSAME_E_OOM;
    HIPCHK(hipMemcpyAsync(c->minraw.p, mr.data(), mr.size() * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->minlen.p, ml.data(), ml.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->minident.p, mi.data(), mi.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));   // host vectors die here
    c->tab_valid = true;
    c->tab_min_e = p->min_e; c->tab_cov = p->min_coverage; c->tab_id = p->min_identity;
    c->tab_L = L; c->tab_ymax = ymax; c->tab_xmax = xmax;
    return 0;
}

// IMSAME_DEBUG_TIMELINE=1: every lane's seed scans and NW launches on the
// call's common clock, printed to stderr when the call ends (diagnostics)
static bool timeline_on() {
    static std::once_flag f;
    static bool on = false;
    std::call_once(f, [] { const char *e = getenv("IMSAME_DEBUG_TIMELINE"); on = e && atoi(e); });
    return on;
}
static void timeline_print(const std::vector<imsame_ctx *> &L) {
    for (size_t k = 0; k < L.size(); ++k) {
        for (const auto &e : L[k]->tl)
            fprintf(stderr, "[timeline] lane %zu %c round %d n %u %.3f %.3f\n", k, e.kind, e.round, e.n, e.a, e.b);
        L[k]->tl.clear();
    }
}

struct NwPlan { int G, GPW, xcap, xstride, steps, nstr, k; bool pk, last4, two, lng, lp, np; size_t lds; unsigned blocks, max_blocks;
                uint32_t slot_words;   // np: bitmap words per XCD partition (arena slots = 8 x 32 x slot_words)
                uint64_t tb_dw, ck_dw, bnd_dw; int band_w; };

// Long reads take the two-pass nwl_kernel (nwl_kernel.hip) unless the int32
// kernel is forced (IMSAME_FLAG_NW32, or IMSAME_NWL=0 for A/B runs).
static bool nwl_enabled() {
    static std::once_flag f;
    static bool on = true;
    std::call_once(f, [] { const char *e = getenv("IMSAME_NWL"); on = !(e && !atoi(e)); });
    return on;
}
// ... and on packed pairs (nwp_kernel.hip) where the range proof admits the
// launch (IMSAME_NWP=0 keeps the int32 nwl_kernel, for A/B runs)
static bool nwp_enabled() {
    const char *e = getenv("IMSAME_NWP");
    return !(e && !atoi(e));
}

// Rows above its best cell the second nw16 sweep keeps (nw16_kernel.hip).  A
// path longer than that (rare: C2 paths span <= 209 rows) makes its wave redo
// the sweep over 4 bands, then from row 1.  IMSAME_NW_BAND overrides (tests
// use tiny bands to drive the redo path).
static int nw16_band_rows() {
    const char *e = getenv("IMSAME_NW_BAND");
    return e ? std::max(0, atoi(e)) : 200;
}


// Slot strides of the non-persistent arena: the largest packed shape of a
// record cap (reads <= NW_W/2, either column form), so the launches of every
// lane of a call -- whose read lengths differ -- share one layout.
static void np_strides(uint32_t xcap, uint64_t *tb_dw, uint64_t *ck_dw) {
    const NwShape a = nw16_shape(NW_W / 2, xcap, NW16_K), b = nw16_shape(NW_W / 2, xcap, NW16_K5),
                  d = nw16_shape(NW16_K19_YLEN, xcap, NW16_K19), e = nw16_shape(NW16_K3_YMAX, xcap, NW16_K3);
    *tb_dw = std::max(std::max(nw16_tb_words(a), nw16_tb_words(b)), std::max(nw16_tb_words(d), nw16_tb_words(e)));
    *ck_dw = std::max(std::max(nw16_ck_words(a), nw16_ck_words(b)), std::max(nw16_ck_words(d), nw16_ck_words(e)));
}

// Blocks per CU the XCD partitions of a context's slot bitmap hold: the
// largest residency of any packed variant without LDS (LDS only lowers it),
// so every non-persistent launch of the context -- and any two running at
// once, whatever their forms -- numbers its slots the same way.  0: unknown.
static int nw16_np_part_cu(imsame_ctx *c) {
    if (c->np_part_cu >= 0) return c->np_part_cu;
    int m = 0;
    bool ok = true;
    auto q = [&](const void *f) {
        int a = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, f, 256, 0) != hipSuccess || a < 1) ok = false;
        m = std::max(m, a);
    };
    q((const void *)nw16_kernel<NW16_K, false, true>);  q((const void *)nw16_kernel<NW16_K, true, true>);
    q((const void *)nw16_kernel<NW16_K, false, false>); q((const void *)nw16_kernel<NW16_K, true, false>);
    q((const void *)nw16_kernel<NW16_K5, false, true>); q((const void *)nw16_kernel<NW16_K5, true, true>);
    q((const void *)nw16_kernel<NW16_K5, false, false>); q((const void *)nw16_kernel<NW16_K5, true, false>);
    q((const void *)nw16_kernel<NW16_K19, true, true, NW16_K19_OFF>);
    q((const void *)nw16_kernel<NW16_K19, true, false, NW16_K19_OFF>);
    q((const void *)nw16_kernel<NW16_K3, false, true>); q((const void *)nw16_kernel<NW16_K3, true, true>);
    q((const void *)nw16_kernel<NW16_K3, false, false>); q((const void *)nw16_kernel<NW16_K3, true, false>);
    c->np_part_cu = ok ? m : 0;
    return c->np_part_cu;
}

// Columns per lane of a packed launch.  A launch is a queue of tasks (8
// candidates x all rows at K = 10) pulled by one wave per resident slot
// (4 per SIMD); a launch of a few slots' worth (a lane's later rounds, every
// round of an 8-GPU shard) spends most of its time in its last tasks with
// the chip mostly idle.  K = 5 halves a task (4 candidates, each wave half
// the columns per step) and doubles their number, for ~8 % more
// instructions per cell.  Chosen when the launch holds fewer than
// k5_fill x (the chip's K = 10 slots / the lanes running) tasks.
// IMSAME_NW_K=5|10 forces one; IMSAME_NW_K5_FILL sets k5_fill.  Round 3
// measured k5_fill 2 slower (the C2 1/8 shard 21.3-21.5 ms against
// 20.5-20.6, profiles/r3o_*: launches of ~10k candidates share the chip with
// the other lanes' large ones).  Round 5: at 0.3 (below ~3.3k candidates with
// 3 lanes) K = 5 replaces the int32 kernel that ran those launches (plan_nw's
// `small`): alone on the chip a 2000 x 150 launch takes 0.59 / 0.63 / 0.74 ms
// at 128 / 1400 / 4096 candidates against 0.68 / 0.71 / 1.17 (int32) and
// 1.69 / 1.72 / 1.79 (K = 19) (profiles/r5y/nwsmall_r5y.json); the 1/4 shard's
// round-2 launches (~2.9k candidates) went 1.1-1.9 -> 0.8-1.4 ms and the
// shard 29.7 -> 28.8 ms, C2 and the 1/8 shard unchanged (profiles/r5z/).
// Round 6: the 3-column latency form (NW16_K3) takes a lane's launches of
// rounds >= 2 below IMSAME_NW_K3_MAX candidates (reads <= NW16_K3_YMAX; the
// caller checks the range proof for its shape); IMSAME_NW_K=3 forces it.
// Alone on the chip, 2000 x 150 launches take (K = 3 vs 5 columns) 0.38-0.42
// vs 0.50-0.56 ms for one pair, 0.54-0.58 vs 0.62-0.65 ms for 1400 pairs,
// 0.86 vs 0.75 ms for 4096 (profiles/r6a/nwsmall_r6a.json): the default
// bound sits between the last two.
static uint32_t nw16_k3_max() {
    static uint32_t v = [] { const char *e = getenv("IMSAME_NW_K3_MAX"); return e ? (uint32_t)atoi(e) : 2048u; }();
    return v;
}
// the round of the launch being planned / timed: per host thread (a lane,
// or one of a lane's two read pipelines)
static thread_local int t_round = 0;
// align_one: reads with round-1 candidates and round 1b's reads run their
// later rounds as independent pipelines (IMSAME_PIPES=0: joined rounds)
// ... and round 1's launch cut into unpredicted + predicted candidates
// (IMSAME_CUT_WEAK=0: one launch)
static bool cut_weak_on() {
    const char *e = getenv("IMSAME_CUT_WEAK");
    return !(e && !atoi(e));
}
// Measured (profiles/r6e/): C2 (lanes of 333k reads) 100.7-100.8 ms per step
// against 101.3 joined; the 1/8 and 1/4 shards (lanes of 42k / 83k reads)
// 16.2 / 29.0 ms against 15.3 / 27.6 -- there the weak launch and round 1b's
// queue one behind the other on stream_b and B ends last.  So: lanes of >=
// 200k reads (the budget rule's bound, round_policy.h); IMSAME_PIPES=1 / 0
// forces it (read per call: tests compare both forms).
static bool pipes_on(uint64_t n) {
    const char *e = getenv("IMSAME_PIPES");
    return e ? atoi(e) != 0 : n >= 200000;
}
// The second pipeline at high priority (stream_bh): IMSAME_PRIO_B=0 never,
// 1 always, unset: where this lane's previous pipelined call ran more NW
// candidates in the second pipeline than in the first (c->b_prio).  Then
// the weak reads' chain of rounds is the call's critical path and takes the
// wave slots its launches free first, while the first pipeline's big round-1
// launch fills the rest (C3: 350.5 -> 341.5-343.8 ms; at C2 the first
// pipeline's launch is the long one, and priority for the second made it
// 97.0 -> 98.2 ms, profiles/r6p2/).
static bool prio_b(const imsame_ctx *c) {
    const char *e = getenv("IMSAME_PRIO_B");
    return c->stream_bh && (e ? atoi(e) != 0 : c->b_prio);
}
static int nw16_k(imsame_ctx *c, uint32_t ncand, bool rounds) {
    const char *e = getenv("IMSAME_NW_K"), *fe = getenv("IMSAME_NW_K5_FILL"), *f2 = getenv("IMSAME_NW_K5_FILL2");
    const int force = e ? atoi(e) : 0;
    if (force == NW16_K3 || force == NW16_K5 || force == NW16_K) return force;
    if (rounds && t_round >= 2 && ncand <= nw16_k3_max()) return NW16_K3;
    // a lane's launches of rounds >= 2 (IMSAME_NW_K5_FILL2, 1.5: below ~16k
    // candidates with 3 lanes): C2's round-2 launches of ~15.5k candidates
    // run one or two 19-column waves per SIMD, latency-bound; the 5-column
    // form took C2 from 105.8-105.9 to 105.2-105.3 ms per step, the 1/8 shard
    // and C3 unchanged (profiles/r5zt/; 1.5 for every launch, round 1b's
    // included, slowed the 1/8 shard and C3: r5zs/)
    const double fill = t_round >= 2 ? (f2 ? atof(f2) : 1.5) : fe ? atof(fe) : 0.3;
    if (!rounds) return NW16_K;
    const double slots = (double)c->ncu * 4.0 * 4.0 / std::max(1, c->nlanes);
    return (double)ncand / 8.0 < fill * slots ? NW16_K5 : NW16_K;
}

// pk: the packed-pair int16 kernel (nw16_kernel.hip) when the launch fits it
// ylen_mult: every read of the launch has a length that is a multiple of NW16_K
// ylen_uni: the one length of every read of the launch (0: lengths differ)
static int plan_nw(imsame_ctx *c, uint32_t ymax, uint32_t xcap, uint32_t ncand, const imsame_params *p,
                   bool ylen_mult, NwPlan *pl, bool rounds = true, uint32_t ylen_uni = 0) {
    const int wpb = 4;
    // Small launches (the last rounds; every round of a small shard) are
    // latency-bound: one 19-column task is 16 candidates x all rows (~1.6 ms
    // alone on a SIMD).  Rounds 3-4 ran launches below 3000 candidates on the
    // int32 kernel (5 columns per lane, 2 candidates per wave); since round 5
    // the packed kernel's 5-column form takes them (nw16_k: faster alone at
    // every size, profiles/r5y/).  IMSAME_NW_SMALL=N: the int32 kernel below N
    // candidates again.  Results are identical (tests run every kernel).
    const char *se = getenv("IMSAME_NW_SMALL");
    const uint32_t small = (p->flags & IMSAME_FLAG_NW16) || !rounds ? 0u : se ? (uint32_t)atoi(se) : 0u;
    pl->pk = !(p->flags & IMSAME_FLAG_NW32) && ncand >= small && nw16_fits(p->igap, p->egap, xcap, ymax);
    pl->last4 = pl->pk && ylen_mult;
    const char *op = getenv("IMSAME_NW_ONEPASS");
    pl->two = pl->pk && !(p->flags & IMSAME_FLAG_NW16_ONEPASS) && !(op && atoi(op));
    pl->band_w = nw16_band_rows();
    pl->lng = !pl->pk && !(p->flags & IMSAME_FLAG_NW32) && nwl_enabled() && nwl_fits(p->igap, p->egap, ymax);
    if (pl->lng) {                  // steps of a pass-2 band (IMSAME_NWL_BAND: tests use small ones)
        const char *nb = getenv("IMSAME_NWL_BAND");
        pl->band_w = nb ? std::max(1, std::min(NWL_BAND, atoi(nb))) : NWL_BAND_DEF;
    }
    pl->lp = pl->lng && nwp_enabled() && nwp_fits(p->igap, p->egap, xcap, ymax);
    pl->k = pl->pk ? nw16_k(c, ncand, rounds) : 0;
    if (pl->k == NW16_K3) {
        // the latency form: reads <= NW16_K3_YMAX (CK + G <= 64, nw16_fits) whose
        // values fit its wider column count; LAST when the launch's one read
        // length is a multiple of 3 (ylen_mult speaks of NW16_K)
        if (ymax > NW16_K3_YMAX || !nw16_fits(p->igap, p->egap, xcap, ymax, NW16_K3)) pl->k = NW16_K5;
        else pl->last4 = ylen_uni && ylen_uni == ymax && ylen_uni % NW16_K3 == 0;
    }
    if (pl->pk && pl->k == NW16_K && nw16_k19_ok(ylen_uni, ymax, xcap, p)) {
        pl->k = NW16_K19;
        pl->last4 = true;                   // 150 = 8 x 19 - OFF: last column in slot K-1
    }
    const NwShape sh = pl->pk ? nw16_shape(ymax, xcap, pl->k) : pl->lp ? nwp_shape(ymax, xcap)
                     : pl->lng ? nwl_shape(ymax, xcap) : nw_shape(ymax, xcap);
    pl->G = sh.G; pl->GPW = sh.GPW; pl->nstr = sh.nstr; pl->xcap = sh.xcap; pl->xstride = sh.xstride;
    pl->steps = sh.steps;
    pl->tb_dw = pl->pk ? nw16_tb_words(sh) : pl->lp ? nwp_tb_words(sh, ymax) : pl->lng ? nwl_tb_words(sh, ymax) : nw_tb_words(sh);
    pl->ck_dw = pl->two ? nw16_ck_words(sh) : pl->lp ? nwp_ck_words(sh, ymax) : pl->lng ? nwl_ck_words(sh) : 0;
    pl->bnd_dw = pl->lp ? nwp_seam_words(sh, ymax) : pl->lng ? nwl_seam_words(sh) : 3ull * pl->xcap;
    pl->lds = (size_t)wpb * (pl->pk ? nw16_wave_lds(pl->GPW, pl->xstride)
                             : pl->lng ? nwl_wave_lds(pl->xstride) : nw_wave_lds(pl->GPW, pl->xstride));
    int per_cu = 0;
    const bool k5 = pl->k == NW16_K5, k19 = pl->k == NW16_K19, k3 = pl->k == NW16_K3;
    hipError_t oe = pl->lp ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nwp_kernel, wpb * 64, pl->lds)
                  : pl->lng ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nwl_kernel, wpb * 64, pl->lds)
                  : k3 ? (pl->two ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nw16_kernel<NW16_K3, false, true>,
                                                                             wpb * 64, pl->lds)
                                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nw16_kernel<NW16_K3, false, false>,
                                                                             wpb * 64, pl->lds))
                  : k19 ? (pl->two ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                                         &per_cu, nw16_kernel<NW16_K19, true, true, NW16_K19_OFF>, wpb * 64, pl->lds)
                                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                                         &per_cu, nw16_kernel<NW16_K19, true, false, NW16_K19_OFF>, wpb * 64, pl->lds))
                  : pl->two ? (k5 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nw16_kernel<NW16_K5, false, true>, wpb * 64, pl->lds)
                                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nw16_kernel<NW16_K, false, true>, wpb * 64, pl->lds))
                  : pl->pk ? (k5 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nw16_kernel<NW16_K5, false, false>, wpb * 64, pl->lds)
                                 : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nw16_kernel<NW16_K, false, false>, wpb * 64, pl->lds))
                  : (pl->nstr > 1)
                      ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nw_kernel<true>, wpb * 64, pl->lds)
                      : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, nw_kernel<false>, wpb * 64, pl->lds);
    if (oe != hipSuccess || per_cu < 1) per_cu = 1;
    // Non-persistent packed launches (one wave per task, arena slots from a
    // per-XCD free bitmap): waves leave as their tasks end, so other lanes'
    // seed scans and small kernels get wave slots during a long launch
    // instead of after its last task (a persistent wave holds its slot until
    // the queue is empty).  The partitions must hold the kernel's full
    // residency, so per_cu is the true occupancy here.
    pl->np = pl->pk && rounds && nw_xcc_check(c) && nw16_np_part_cu(c) > 0;
    int part_cu = per_cu;                   // np: blocks per CU the XCD partitions hold
    if (pl->np) {
        // One slot layout for both column forms: round 1b runs two packed
        // launches of a lane at once (align_one), possibly of different
        // forms, on one arena and bitmap.  Strides of the larger form;
        // partitions for the larger residency without LDS (LDS only lowers it).
        part_cu = nw16_np_part_cu(c);
        uint64_t tb_dw = 0, ck_dw = 0;
        np_strides(xcap, &tb_dw, &ck_dw);
        const uint32_t words = (uint32_t)((((uint64_t)c->ncu / 8) * part_cu * wpb + 31) / 32);
        const uint64_t ns = (uint64_t)8 * 32 * words;
        // the arena np_prepare actually holds (it skips the allocation when
        // free HBM is short, e.g. after a long-read call grew c->tb): a plan
        // is non-persistent only if its slots exist, so two launches planned
        // np (round 1b) never fall back to one persistent arena together
        const imsame_ctx *ao = c->np_owner ? c->np_owner : c;
        if (part_cu < per_cu || ao->np_tb.cap < ns * tb_dw * 4 || ao->np_ck.cap < ns * ck_dw * 4 ||
            ao->slotbits.cap < (uint64_t)8 * words * 4)
            pl->np = false;
        else { pl->tb_dw = tb_dw; pl->ck_dw = ck_dw; }
    }
    if (!pl->np) { per_cu = std::min(per_cu, 8); part_cu = per_cu; }
    const uint32_t cpw = (pl->pk || pl->lp) ? 2 * pl->GPW : pl->GPW;    // candidates per wave pull
    const uint64_t waves_needed = (ncand + cpw - 1) / cpw;
    pl->slot_words = (uint32_t)((((uint64_t)c->ncu / 8) * part_cu * wpb + 31) / 32);
    pl->blocks = (unsigned)std::max<uint64_t>(1, pl->np ? (waves_needed + wpb - 1) / wpb
                                                         : std::min<uint64_t>((uint64_t)c->ncu * per_cu, (waves_needed + wpb - 1) / wpb));
    // Traceback arena: one slot per resident wave.  Long reads against long
    // records (C5w, 10 kbp x 12 kbp = 99 MB per slot) would ask for more than
    // the card holds at full residency; the kernel pulls candidates from a
    // queue, so fewer blocks finish the same work.  Budget: what is free
    // (counting the arena already held) less 8 GB of headroom -- the 288 GB
    // of HBM are there to keep waves resident.
    const uint64_t per_block = (uint64_t)wpb * (pl->tb_dw * 4 + pl->ck_dw * 4 + pl->bnd_dw * 4);
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = 0;
    const uint64_t held = c->tb.cap + c->bnd.cap + c->ck.cap;
    const uint64_t avail = fr + held, headroom = 8ull << 30;
    const uint64_t budget = avail > 2 * headroom ? avail - headroom : avail / 2;
    const uint64_t fit = budget / per_block;
    if (fit < 1) return IMSAME_E_OOM;
    if (pl->np && (uint64_t)8 * 32 * pl->slot_words > fit * wpb) {   // arena short of the residency
        pl->np = false;
        pl->blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)c->ncu * std::min(per_cu, 8),
                                                                        (waves_needed + wpb - 1) / wpb));
    }
    if (pl->np) {                           // the arena holds 8 x 32 x slot_words slots
        pl->max_blocks = (unsigned)(((uint64_t)8 * 32 * pl->slot_words + wpb - 1) / wpb);
        return 0;
    }
    if (pl->blocks > fit) pl->blocks = (unsigned)fit;
    // the arena is sized for a full-residency launch of this shape, so the
    // launches of later rounds (fewer or more candidates) reuse it instead of
    // reallocating up to hundreds of GB each round
    pl->max_blocks = (unsigned)std::min<uint64_t>((uint64_t)c->ncu * per_cu, fit);
    if (pl->max_blocks < pl->blocks) pl->max_blocks = pl->blocks;
    return 0;
}

// end of an NW launch enqueued by launch_nw on queue qi: its duration and
// its interval on the call's common clock
static int nw_launch_done(imsame_ctx *c, int qi, uint32_t n, double *ms) {
    hipEvent_t e0 = qi ? c->evb0 : c->ev0, e1 = qi ? c->evb1 : c->ev1;
    if (wait_block())                                              // recorded behind e1 (launch_nw)
        if (int r = ev_wait(c->evw[qi ? 1 : 0][1])) return r;
    HIPCHK(hipEventSynchronize(e1));
    float f = 0;
    HIPCHK(hipEventElapsedTime(&f, e0, e1));
    *ms = f;
    if (c->origin) {
        float a = 0, b = 0;
        if (hipEventElapsedTime(&a, c->origin, e0) == hipSuccess && hipEventElapsedTime(&b, c->origin, e1) == hipSuccess) {
            std::lock_guard<std::mutex> g(c->iv_mu);
            c->nw_iv.push_back({a, b});
            if (timeline_on()) c->tl.push_back({'N', t_round, n, a, b});
        }
    }
    return 0;
}

// The shared arena of non-persistent packed launches (np_strides, slot
// partitions of nw16_np_part_cu), allocated before a call's lanes start:
// growing it while launches run would free memory in use, and hipFree waits
// for the whole device.  Skipped (launches stay persistent) where the
// probe failed or the free memory less 8 GB cannot hold it.
static int np_prepare(imsame_ctx *o, uint32_t xcap) {
    if (!nw_xcc_check(o) || nw16_np_part_cu(o) < 1) return 0;
    // test hook: behave as if free HBM could not hold the arena (the state a
    // long-read call that grew the persistent arena leaves behind)
    if (const char *sk = getenv("IMSAME_DEBUG_NP_SKIP")) if (atoi(sk)) return 0;
    const uint32_t words = (uint32_t)((((uint64_t)o->ncu / 8) * nw16_np_part_cu(o) * 4 + 31) / 32);
    const uint64_t ns = (uint64_t)8 * 32 * words, nbits = (uint64_t)8 * words * 4;
    uint64_t tb_dw = 0, ck_dw = 0;
    np_strides(xcap < 2 ? 2 : xcap, &tb_dw, &ck_dw);
    const uint64_t need_tb = ns * tb_dw * 4, need_ck = ns * ck_dw * 4;
    if (o->np_tb.cap >= need_tb && o->np_ck.cap >= need_ck && o->slotbits.cap >= nbits) return 0;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 0;
    const uint64_t held = o->np_tb.cap + o->np_ck.cap;
    if (fr + held < need_tb + need_ck + (8ull << 30)) return 0;
    hipStream_t s = o->stream;
    if (o->np_tb.ensure(need_tb) || o->np_ck.ensure(need_ck)) { o->np_tb.release(); o->np_ck.release(); return 0; }
    if (o->slotbits.cap < nbits) {               // all free: waves clear their bits as they leave
        if (o->slotbits.ensure(nbits)) return IMSAME_E_OOM;
        HIPCHK(hipMemsetAsync(o->slotbits.p, 0, o->slotbits.cap, s));
    }
    if (poison_on()) {
        if (int rc = o->np_tb.poison(s)) return rc;
        if (int rc = o->np_ck.poison(s)) return rc;
    }
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

// Queue order of a launch's candidates by predicted first row (8-row
// buckets, unpredicted first: launch_nw's own ordering, done ahead of it) into
// the cperm buffer of queue qi, and the number of unpredicted candidates --
// the first *nweak entries -- read back (the stream is synchronized).
static int row_perm(imsame_ctx *c, const int32_t *crow, uint32_t n, uint32_t xcap_pl, int qi, uint32_t *nweak) {
    hipStream_t s = qi ? c->stream_b : c->stream;
    const uint32_t nb = xcap_pl / 8 + 512 / 8 + 2;
    DBuf &cperm = qi ? c->cperm_b : c->cperm, &rhist = qi ? c->rhist_b : c->rhist;
    if (cperm.ensure((uint64_t)n * 4) || rhist.ensure((uint64_t)nb * 8)) return IMSAME_E_OOM;
    uint32_t *hist = rhist.as<uint32_t>(), *cur = hist + nb;
    HIPCHK(hipMemsetAsync(hist, 0, (size_t)nb * 4, s));
    row_hist_kernel<<<std::min(nblk(n, 256), ROW_BLOCKS), 256, 0, s>>>(crow, n, nb, hist);
    row_scan_kernel<<<1, 1024, 0, s>>>(hist, nb, cur);
    row_scatter_kernel<<<std::min(nblk(n, 256), ROW_BLOCKS), 256, 0, s>>>(crow, n, nb, cur, cperm.as<uint32_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(nweak, hist, 4, hipMemcpyDeviceToHost, s));
    LANE_SYNC(c, s);
    return 0;
}

static int launch_nw(imsame_ctx *c, NwPlan &pl, const uint32_t *cread, const uint32_t *csid, uint32_t n,
                     imsame_read_result *outp, int64_t ig, int64_t eg, const imsame_params *p, uint32_t ymax,
                     uint32_t xmax, uint32_t *work, const uint8_t *dbp, const uint64_t *dbs, const uint8_t *qp,
                     const uint64_t *qs, uint32_t paths_cap, double *ms, const int32_t *crow = nullptr, int qi = 0,
                     bool wait = true, const uint32_t *perm_in = nullptr) {
    // perm_in: the queue order is given (row_perm; the candidates are
    // perm_in[0 .. n)), crow their predicted rows
    // qi 1: round 1b's stream; wait false: enqueue only (nw_launch_done)
    hipStream_t s = qi ? c->stream_b : c->stream;
    hipEvent_t e0 = qi ? c->evb0 : c->ev0, e1 = qi ? c->evb1 : c->ev1;
    const uint64_t tb_dw = pl.tb_dw;
    // fewer resident waves if the arena cannot be had (the queue still drains)
    const uint64_t per_slot = tb_dw * 4, bnd_slot = pl.bnd_dw * 4, ck_slot = pl.ck_dw * 4;
    imsame_ctx *ao = c->np_owner ? c->np_owner : c;     // the shared arena (np_prepare)
    if (pl.np) {                                 // every slot of the 8 partitions, and their bitmap
        const uint64_t ns = (uint64_t)pl.max_blocks * 4, nbits = (uint64_t)8 * pl.slot_words * 4;
        if (ao->np_tb.cap < ns * per_slot || ao->np_ck.cap < ns * ck_slot || ao->slotbits.cap < nbits) {
            pl.np = false;                       // not prepared for this shape: persistent on this lane's
            pl.blocks = (unsigned)std::min<uint64_t>((uint64_t)c->ncu * 8, pl.blocks);
        }
    }
    if (!pl.np) {
        if (c->tb.cap < (uint64_t)pl.blocks * 4 * per_slot)       // grow once to this shape's full residency
            (void)c->tb.ensure((uint64_t)pl.max_blocks * 4 * per_slot);
        if (ck_slot && c->ck.cap < (uint64_t)pl.blocks * 4 * ck_slot)
            (void)c->ck.ensure((uint64_t)pl.max_blocks * 4 * ck_slot);
        while (c->tb.ensure((uint64_t)pl.blocks * 4 * per_slot) || c->bnd.ensure((uint64_t)pl.blocks * 4 * bnd_slot + 64) ||
               (ck_slot && c->ck.ensure((uint64_t)pl.blocks * 4 * ck_slot))) {
            if (pl.blocks == 1) return IMSAME_E_OOM;
            pl.blocks = (pl.blocks + 1) / 2;
        }
    }
    if (poison_on() && !pl.np) {                 // slots hold nothing from earlier launches (the shared
        const DBuf *scr[] = {&c->tb, &c->ck, &c->bnd};          // arena: at np_prepare)
        for (const DBuf *b : scr)
            if (int rc = b->poison(s)) return rc;
    }
    NwLaunch P;
    memset(&P, 0, sizeof P);
    P.db = dbp; P.db_start = dbs; P.q = qp; P.q_start = qs;
    P.cand_read = cread; P.cand_sid = csid; P.n_cand = n;
    P.igap = (int32_t)ig; P.egap = (int32_t)eg;
    P.G = pl.G; P.GPW = pl.GPW; P.xcap = pl.xcap; P.xstride = pl.xstride; P.steps = pl.steps;
    P.tb = pl.np ? ao->np_tb.as<uint32_t>() : c->tb.as<uint32_t>(); P.tb_wave_dw = tb_dw;
    P.bnd = c->bnd.as<int32_t>(); P.bnd_wave = pl.bnd_dw;
    P.minlen = c->minlen.as<uint32_t>(); P.n_minlen = ymax + 1;
    P.minident = c->minident.as<uint32_t>(); P.n_minident = xmax + ymax + 2;
    P.counter = work;
    P.out = outp;
    uint64_t *ctr = c->ctr.as<uint64_t>();
    P.paths = c->paths.as<uint32_t>(); P.paths_cap = paths_cap;
    P.paths_used = (uint32_t *)(ctr + C_PATHS); P.want_paths = p->want_paths;
    P.flags = (uint32_t *)(ctr + C_FLAGS);
    P.ck = !(pl.two || pl.lng) ? nullptr : pl.np ? ao->np_ck.as<uint32_t>() : c->ck.as<uint32_t>();
    P.ck_wave_dw = pl.ck_dw;
    P.band_w = pl.band_w; P.redo = (uint32_t *)(ctr + C_REDO); P.win = (uint32_t *)(ctr + C_WIN);
    P.prof = getenv("IMSAME_NW_PROF") ? (unsigned long long *)(ctr + C_PROF) : nullptr;
    P.slot_bits = pl.np ? ao->slotbits.as<uint32_t>() : nullptr; P.slot_words = pl.slot_words;
    HIPCHK(hipMemsetAsync(work, 0, 4, s));
    HIPCHK(hipEventRecord(e0, s));               // the launch's time includes its ordering
    auto win_params = [&] {
        const char *wu = getenv("IMSAME_NW_WIN_UP"), *wd = getenv("IMSAME_NW_WIN_DOWN");
        P.win_up = wu ? atoi(wu) : NW16_WIN_UP; P.win_down = wd ? atoi(wd) : NW16_WIN_DOWN;
        const char *wb = getenv("IMSAME_NW_WIN_BOTTOM");
        P.win_bottom = wb ? atoi(wb) : NW16_WIN_BOTTOM;
    };
    if (perm_in) {
        P.perm = perm_in;
        if (crow && pl.two) { P.cand_row = crow; win_params(); }
    } else if (crow && pl.two && n >= 64) {
        // queue order by predicted row (first-sweep traceback windows)
        const uint32_t nb = ((uint32_t)pl.xcap + 512) / 8 + 2;
        DBuf &cperm = qi ? c->cperm_b : c->cperm, &rhist = qi ? c->rhist_b : c->rhist;
        if (cperm.ensure((uint64_t)n * 4) || rhist.ensure((uint64_t)nb * 8)) return IMSAME_E_OOM;
        uint32_t *hist = rhist.as<uint32_t>(), *cur = hist + nb;
        HIPCHK(hipMemsetAsync(hist, 0, (size_t)nb * 4, s));
        row_hist_kernel<<<std::min(nblk(n, 256), ROW_BLOCKS), 256, 0, s>>>(crow, n, nb, hist);
        row_scan_kernel<<<1, 1024, 0, s>>>(hist, nb, cur);
        row_scatter_kernel<<<std::min(nblk(n, 256), ROW_BLOCKS), 256, 0, s>>>(crow, n, nb, cur, cperm.as<uint32_t>());
        HIPCHK(hipGetLastError());
        P.perm = cperm.as<uint32_t>(); P.cand_row = crow;
        const char *wu = getenv("IMSAME_NW_WIN_UP"), *wd = getenv("IMSAME_NW_WIN_DOWN");
        P.win_up = wu ? atoi(wu) : NW16_WIN_UP; P.win_down = wd ? atoi(wd) : NW16_WIN_DOWN;
        const char *wb = getenv("IMSAME_NW_WIN_BOTTOM");
        P.win_bottom = wb ? atoi(wb) : NW16_WIN_BOTTOM;
    }
    const bool k5 = pl.k == NW16_K5;
    if (pl.lp) {
        P.rlim = (int32_t)nwp_rlim(ig, eg, (uint64_t)pl.xcap, ymax);
        const char *ns = getenv("IMSAME_NWP_S");          // tests: a tiny spread drives the int32 fallback
        P.nwp_s = ns ? atoi(ns) : 0;
        P.fbk = (uint32_t *)(ctr + C_FBK);
    }
    if (pl.lp)                         nwp_kernel<<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.lng)                   nwl_kernel<<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.k == NW16_K19 && pl.two) nw16_kernel<NW16_K19, true, true, NW16_K19_OFF><<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.k == NW16_K19)         nw16_kernel<NW16_K19, true, false, NW16_K19_OFF><<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.k == NW16_K3 && pl.two && pl.last4) nw16_kernel<NW16_K3, true, true><<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.k == NW16_K3 && pl.two) nw16_kernel<NW16_K3, false, true><<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.k == NW16_K3 && pl.last4) nw16_kernel<NW16_K3, true, false><<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.k == NW16_K3)          nw16_kernel<NW16_K3, false, false><<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.two && pl.last4 && k5) nw16_kernel<NW16_K5, true, true><<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.two && k5)             nw16_kernel<NW16_K5, false, true><<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.pk && pl.last4 && k5)  nw16_kernel<NW16_K5, true, false><<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.pk && k5)              nw16_kernel<NW16_K5, false, false><<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.two && pl.last4)       nw16_kernel<NW16_K, true, true><<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.two)                   nw16_kernel<NW16_K, false, true><<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.pk && pl.last4)        nw16_kernel<NW16_K, true, false><<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.pk)                    nw16_kernel<NW16_K, false, false><<<pl.blocks, 256, pl.lds, s>>>(P);
    else if (pl.nstr > 1) nw_kernel<true><<<pl.blocks, 256, pl.lds, s>>>(P);
    else                  nw_kernel<false><<<pl.blocks, 256, pl.lds, s>>>(P);
    HIPCHK(hipEventRecord(e1, s));
    if (wait_block()) HIPCHK(hipEventRecord(c->evw[qi ? 1 : 0][1], s));
    HIPCHK(hipGetLastError());
    POISON_SYNC(s, pl.pk ? "nw16_kernel" : pl.lp ? "nwp_kernel" : pl.lng ? "nwl_kernel" : "nw_kernel", c);
    return wait ? nw_launch_done(c, qi, n, ms) : 0;
}

static int paths_setup(imsame_ctx *c, const imsame_params *p, uint64_t paths_cap, uint32_t *cap32) {
    *cap32 = 0;
    c->paths_cap_dev = 0;
    if (p->want_paths) {
        *cap32 = (uint32_t)std::min<uint64_t>(paths_cap, 0xFFFFFFF0u);
        if (c->paths.ensure((uint64_t)*cap32 * 4 + 16)) return IMSAME_E_OOM;
        c->paths_cap_dev = *cap32;
    }
    return 0;
}

// grow the device path arena to `need` entries, keeping entries [0, keep)
static int paths_grow(imsame_ctx *c, uint64_t keep, uint64_t need) {
    if (need > 0xFFFFFFF0ull) return IMSAME_E_OOM;                  // u32 path offsets
    if (need <= c->paths_cap_dev) return 0;
    DBuf nb;
    if (nb.ensure(need * 4 + 16)) return IMSAME_E_OOM;
    if (keep) HIPCHK(hipMemcpyAsync(nb.p, c->paths.p, keep * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->paths.release();
    c->paths.p = nb.p; c->paths.cap = nb.cap;
    nb.p = nullptr; nb.cap = 0;
    c->paths_cap_dev = need;
    return 0;
}

// Accepted reads whose path did not fit the device arena (path_off ~0,
// path_len = entries needed).  NW + backtracking is a pure function of
// (record, read), so re-running exactly those pairs
// with room for their paths gives the same rows plus the paths -- instead of
// re-running the whole alignment.  Appends after entry *used.
static int rewalk_lost(imsame_ctx *c, const imsame_params *p, uint64_t read_from, uint32_t n,
                       imsame_read_result *res, uint32_t ymax, uint32_t xcap, uint32_t ycap, uint32_t short_y,
                       uint64_t *used, imsame_stats *st) {
    std::vector<uint32_t> rd[2], sid[2], kk[2];
    uint64_t need = 0;
    for (uint32_t k = 0; k < n; ++k) {
        if (res[k].status != 1 || res[k].path_off != 0xFFFFFFFFu) continue;
        const int cl = res[k].ylen <= short_y ? 0 : 1;
        rd[cl].push_back((uint32_t)(read_from + k)); sid[cl].push_back((uint32_t)res[k].db_seq); kk[cl].push_back(k);
        need += res[k].path_len;
    }
    if (rd[0].empty() && rd[1].empty()) return 0;      // only discarded speculative candidates lost theirs
    const uint64_t base = *used, cap = base + need + 16;
    int rc = paths_grow(c, base, cap);
    if (rc) return rc;
    hipStream_t s = c->stream;
    uint64_t *ctr = c->ctr.as<uint64_t>();
    const uint64_t zero = 0;
    HIPCHK(hipMemcpyAsync(ctr + C_PATHS, &base, 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(ctr + C_FLAGS, &zero, 8, hipMemcpyHostToDevice, s));
    for (int cl = 0; cl < 2; ++cl) {
        const uint32_t m = (uint32_t)rd[cl].size();
        if (!m) continue;
        HIPCHK(hipMemcpyAsync(c->cread.p, rd[cl].data(), (uint64_t)m * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(c->csid.p, sid[cl].data(), (uint64_t)m * 4, hipMemcpyHostToDevice, s));
        NwPlan pl;
        if ((rc = plan_nw(c, cl ? ycap : short_y, xcap, m, p, c->q_len_mult, &pl, true, c->q_len_uni))) return rc;
        double ms = 0;
        rc = launch_nw(c, pl, c->cread.as<uint32_t>(), c->csid.as<uint32_t>(), m, c->cout.as<imsame_read_result>(),
                       p->igap, p->egap, p, ymax, xcap, (uint32_t *)(ctr + C_WORK), c->db.as<uint8_t>(),
                       c->db_start.as<uint64_t>(), dev_q(c), dev_qs(c), (uint32_t)cap, &ms);
        if (rc) return rc;
        std::vector<imsame_read_result> o(m);
        HIPCHK(hipMemcpyAsync(o.data(), c->cout.p, (uint64_t)m * 64, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        for (uint32_t j = 0; j < m; ++j) {
            imsame_read_result &r = res[kk[cl][j]];
            if (o[j].status != 1 || o[j].path_off == 0xFFFFFFFFu || o[j].db_seq != r.db_seq || o[j].score != r.score ||
                o[j].length != r.length || o[j].identities != r.identities || o[j].head_x != r.head_x)
                return IMSAME_E_STATE;                                   // NW is pure: cannot differ
            r.path_off = o[j].path_off; r.path_len = o[j].path_len;
        }
        st->n_rewalk += m;
    }
    uint64_t u = 0;
    HIPCHK(hipMemcpyAsync(&u, ctr + C_PATHS, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    *used = (uint32_t)u;
    return 0;
}

// one lane's alignment of reads [read_from, read_to) (arguments checked)
// Blocks of an update launch (update_kernel strides over the candidates):
// few waves, so a launch queued while other lanes' NW waves hold the chip
// starts as soon as a handful of slots free up.  IMSAME_UPD_BLOCKS overrides.
static unsigned upd_blocks() {
    static unsigned v = [] { const char *e = getenv("IMSAME_UPD_BLOCKS"); return e ? std::max(1, atoi(e)) : 64; }();
    return v;
}
// ... and of a seed launch (the scan kernels stride over the reads' groups):
// unlimited unless IMSAME_SEED_BLOCKS is set
static unsigned seed_blocks() {
    static unsigned v = [] { const char *e = getenv("IMSAME_SEED_BLOCKS"); return e ? std::max(1, atoi(e)) : 1u << 30; }();
    return v;
}

static int align_one(imsame_ctx *c, uint64_t read_from, uint64_t read_to, uint64_t n_threads_semantic,
                     const imsame_params *p, imsame_read_result *res, uint32_t *paths, uint64_t paths_cap,
                     uint64_t *paths_used, imsame_stats *stats) {
    const double t_start = now_ms();
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const uint32_t n = (uint32_t)(read_to - read_from);
    // the second pipeline's stream for this call (prio_b), back at return
    struct StreamSwap {
        imsame_ctx *c; bool on;
        ~StreamSwap() { if (on) std::swap(c->stream_b, c->stream_bh); }
    } swap_b{c, pipes_on(n) && prio_b(c)};
    if (swap_b.on) std::swap(c->stream_b, c->stream_bh);
    // this lane's bases (and the 16-byte chunk loads' reach past its last read)
    if (int rq = query_wait(c, s, hqs(c, read_to) + 64)) return rq;
    imsame_stats st;
    memset(&st, 0, sizeof st);
    st.n_reads = n;
    st.err_read = ~0ull;
    st.lanes = 1;
    if (paths_used) *paths_used = 0;
    c->paths_n = 0; c->paths_on_host = false;
    // shapes
    uint32_t ymax = 0;
    ymax = (uint32_t)range_ymax(c, read_from, read_to);
    const uint32_t xcap = (uint32_t)std::min<uint64_t>(c->max_rec, p->max_read_size);
    const uint32_t ycap = (uint32_t)std::min<uint64_t>(ymax, p->max_read_size);
    if (!imsame_gaps_in_range(p->igap, p->egap, xcap, ycap)) return IMSAME_E_RANGE;
    if (std::max(xcap, ycap) > 0x3FFF) return IMSAME_E_ARG;       // 14-bit traceback coordinates
    int rc = build_tables(c, p, ymax, xcap);
    if (rc) return rc;
    // device path arena: what the caller offers, or what the last call needed per read
    uint32_t pcap = 0;
    uint64_t want_cap = std::max<uint64_t>(std::max<uint64_t>(paths_cap, 2ull * n + 1024),
                                           (uint64_t)(c->paths_hint * 1.25 * n) + 1024);
    if (const char *pc = getenv("IMSAME_DEV_PATHS_CAP")) want_cap = strtoull(pc, nullptr, 10);   // test hook
    if ((rc = paths_setup(c, p, want_cap, &pcap))) return rc;
    if (n == 0) { if (stats) *stats = st; return IMSAME_OK; }
    // the rounds' policy (round_policy.h, shared with the CPU emulator):
    // list capacity, speculation, budgets, scan group sizes, round 1b
    const uint32_t short_y = std::min<uint32_t>(ycap, NW_W / 2);
    const RoundPolicy RP = RoundPolicy::make(n, ycap, short_y, c->nlanes);
    const uint64_t ccap = RP.ccap;
    if (c->res.ensure((uint64_t)n * 64) || c->cur_p.ensure((uint64_t)n * 8) || c->cur_h.ensure((uint64_t)n * 4) ||
        c->memo.ensure((uint64_t)n * 4 * MEMO) || c->nmemo.ensure(n) || c->rstat.ensure(n) ||
        c->act0.ensure((uint64_t)n * 4) || c->act1.ensure((uint64_t)n * 4) || c->act2.ensure((uint64_t)n * 4) ||
        c->act3.ensure((uint64_t)n * 4) ||
        c->cread.ensure(ccap * 4) || c->csid.ensure(ccap * 4) ||
        c->cout.ensure(ccap * 64) || c->cbase.ensure((uint64_t)n * 4) ||
        c->ccnt.ensure((uint64_t)n * 4) || c->perr.ensure((uint64_t)n * 4) || c->crow.ensure(ccap * 4))
        return IMSAME_E_OOM;
    // the long-read class (ylen > short_y) only where this call has such reads
    // (72 B per list entry: ~1.3 KB per read of a short-read lane otherwise)
    if (ycap > short_y && (c->cread2.ensure(ccap * 4) || c->csid2.ensure(ccap * 4) || c->cout2.ensure(ccap * 64)))
        return IMSAME_E_OOM;
    if (poison_on()) {                        // this call's scratch holds nothing it may read
        const DBuf *scr[] = {&c->res, &c->cur_p, &c->cur_h, &c->memo, &c->nmemo, &c->rstat, &c->act0, &c->act1, &c->act2,
                             &c->act3,
                             &c->cread, &c->csid, &c->cread2, &c->csid2, &c->cout, &c->cout2, &c->cbase, &c->ccnt,
                             &c->perr, &c->crow, &c->cperm, &c->rhist, &c->cperm_b, &c->rhist_b, &c->paths, &c->tb,
                             &c->ck, &c->bnd};
        for (const DBuf *b : scr)
            if ((rc = b->poison(s))) return rc;
    }
    // predicted rows for the packed kernel's first-sweep traceback windows
    int32_t *crow = RP.window ? c->crow.as<int32_t>() : nullptr;
    const uint8_t *qd = dev_q(c);
    const uint64_t *qsd = dev_qs(c);
    uint64_t *ctr = c->ctr.as<uint64_t>();
    HIPCHK(hipMemsetAsync(ctr, 0, C_NSLOTS * 8, s));
    const unsigned long long errinit = ~0ull;
    HIPCHK(hipMemcpyAsync(ctr + C_ERR, &errinit, 8, hipMemcpyHostToDevice, s));
    // This lane's packed query words (seed_kernel.hip:pk_word; queued after
    // the counters' reset: the packing flags a byte that is not ACGT in
    // C_FLAGS): the words from QPAD bases before its first read to the end of
    // its last part.  Each lane
    // packs its own on its stream as its parts arrive (packing in the upload
    // delayed every lane: the upload's kernels waited for free CUs behind NW
    // waves, profiles/r5t/); neighbouring lanes both write the few words where
    // their reaches meet, with the same values.
    // Words are packed only where all 16 of their bytes are in HBM (below the
    // end of the part waited for): a word at the edge of a part that is still
    // copying would get garbage in the slots a neighbouring lane reads.
    {
        const uint64_t b0 = hqs(c, read_from), b1 = hqs(c, read_to) + 64;
        uint64_t pe = c->qb_end;                          // end of the part query_wait waited for
        for (size_t k = 0; k + 1 < c->q_part_end.size(); ++k)
            if (c->q_part_end[k] >= b1) { pe = c->q_part_end[k]; break; }
        const uint64_t w0 = std::max(c->qw_base, (b0 > QPAD ? b0 - QPAD : 0) / 16);
        const uint64_t w1 = pe == c->qb_end ? c->qw_end : std::min(c->qw_end, pe / 16);
        if (w1 > w0)
            pack2_kernel<<<gsblk(w1 - w0, 256), 256, 0, s>>>(dev_q(c), (int64_t)c->q_base, (int64_t)c->qb_end,
                                                             (uint32_t *)dev_qw(c), w0, w1,
                                                             (unsigned long long *)(ctr + C_FLAGS),
                                                             (int64_t)c->qb_end - 64);      // the zero padding
                                                                                            // (set_query_range_async)
        HIPCHK(hipGetLastError());
    }
    InitLaunch I = {qsd, read_from, n, c->res.as<imsame_read_result>(), c->cur_p.as<uint64_t>(),
                    c->cur_h.as<uint32_t>(), c->nmemo.as<uint8_t>(), c->rstat.as<uint8_t>(), c->act0.as<uint32_t>()};
    init_kernel<<<nblk(n, 256), 256, 0, s>>>(I);
    POISON_SYNC(s, "init_kernel", c);
    HIPCHK(hipGetLastError());
    st.ms_setup = now_ms() - t_start;

    // (round 1b runs under IMSAME_DEBUG_POISON too: the poisoned suite must
    // run the concurrent path -- two streams on the shared arena, slot bitmap,
    // C_PATHS / C_FLAGS counters; POISON_SYNC waits for one stream only)
    // (with predicted traceback windows, round 1's launch is ordered by row;
    // round 1b's candidates carry no prediction and keep their order)
    uint32_t nact = n;
    uint32_t *act = c->act0.as<uint32_t>(), *nxt = c->act1.as<uint32_t>();
    while (nact) {
        st.rounds++;
        c->cur_round = t_round = (int)st.rounds;
        HIPCHK(hipMemsetAsync(ctr + C_NCAND, 0, 7 * 8, s));     // NCAND, NCAND2, NNEXT, (1b) NCANDB, NCAND2B, NNEXT2, WORKB
        SeedLaunch S;
        S.db = c->db.as<uint8_t>(); S.db_start = c->db_start.as<uint64_t>(); S.n_db = c->n_db; S.db_len = c->db_len;
        S.dbw = c->dbw.as<uint32_t>(); S.qw = dev_qw(c);
        S.q = qd; S.q_start = qsd; S.n_q = c->n_q; S.q_len = c->q_len;
        S.qs_lo = c->q_lo; S.qs_lo_first = c->q_lo_first;
        S.off = c->off.as<uint64_t>(); S.ent = c->ent.as<uint2>(); S.ent_abs = c->ent_abs;
        S.active = act; S.n_active = nact;
        S.read_from = read_from;
        S.T = n_threads_semantic ? n_threads_semantic : 1;
        S.rpt = (uint64_t)floorl((long double)c->n_q / (long double)S.T);     // IMSAME.c:414
        S.cur_p = c->cur_p.as<uint64_t>(); S.cur_h = c->cur_h.as<uint32_t>(); S.memo = c->memo.as<uint32_t>();
        S.nmemo = c->nmemo.as<uint8_t>(); S.rstat = c->rstat.as<uint8_t>();
        S.minraw = c->minraw.as<uint64_t>(); S.n_minraw = ymax + 1;
        S.max_rs = p->max_read_size; S.short_ylen = short_y; S.max_rec = c->max_rec;
        const uint32_t rnd = (uint32_t)st.rounds;
        S.spec = RP.spec(rnd, nact);
        S.spec_weak = RP.spec_weak;
        S.budget = RP.budget(rnd);
        S.next = nxt; S.nnext = (uint32_t *)(ctr + C_NNEXT);
        S.cbase = c->cbase.as<uint32_t>(); S.ccnt = c->ccnt.as<uint32_t>(); S.perr = c->perr.as<uint32_t>();
        S.cread = c->cread.as<uint32_t>(); S.csid = c->csid.as<uint32_t>(); S.ncand = (uint32_t *)(ctr + C_NCAND);
        S.crow = crow; S.weak_rows = RP.weak_rows;
        S.cread2 = c->cread2.as<uint32_t>(); S.csid2 = c->csid2.as<uint32_t>(); S.ncand2 = (uint32_t *)(ctr + C_NCAND2);
        S.err = (unsigned long long *)(ctr + C_ERR); S.nhits = (unsigned long long *)(ctr + C_HITS);
        S.nwork = (unsigned long long *)(ctr + C_SWORK);
        S.dbg = getenv("IMSAME_DEBUG_ROUNDS") ? (unsigned long long *)(ctr + C_DBG) : nullptr;
        if (S.dbg) HIPCHK(hipMemsetAsync(S.dbg, 0, 8 * 8, s));
        S.wcap = c->use_wcap ? c->wcap.as<uint64_t>() : nullptr;
        S.wstart = c->use_wstart ? c->wstart.as<uint64_t>() : nullptr;
        S.minlen = c->minlen.as<uint32_t>(); S.n_minlen = ymax + 1;
        S.minident = c->minident.as<uint32_t>(); S.n_minident = xcap + ymax + 2;
        auto seed_launch = [&](const SeedLaunch &SL, uint32_t na, hipStream_t ss, hipEvent_t e0, hipEvent_t e1,
                               uint32_t rr = 0) -> int {
            const int L = RP.pick_L(rr ? rr : rnd, na);
            // (IMSAME_SEED_BLOCKS: at most this many blocks, the kernels stride)
            auto sb = [&](uint64_t lanes) { return std::min<unsigned>(nblk(lanes, 256), seed_blocks()); };
            HIPCHK(hipEventRecord(e0, ss));
            if (SL.ent_abs) {
                if (L >= 64)      seed_group_kernel<64, SPEC_BIG, true><<<sb((uint64_t)na * 64), 256, SEED_LDS_BLOCK(64, SPEC_BIG), ss>>>(SL);
                else if (L >= 16) seed_group_kernel<16, SPEC_MAX, true><<<sb((uint64_t)na * 16), 256, SEED_LDS_BLOCK(16, SPEC_MAX), ss>>>(SL);
                else if (L >= 4)  seed_group_kernel<4, SPEC_MAX, true><<<sb((uint64_t)na * 4), 256, SEED_LDS_BLOCK(4, SPEC_MAX), ss>>>(SL);
                else if (L >= 2)  seed_group_kernel<2, SPEC_MAX, true><<<sb((uint64_t)na * 2), 256, SEED_LDS_BLOCK(2, SPEC_MAX), ss>>>(SL);
                else              seed_kernel<true><<<sb(na), 256, 0, ss>>>(SL);
            } else {
                if (L >= 64)      seed_group_kernel<64, SPEC_BIG, false><<<sb((uint64_t)na * 64), 256, SEED_LDS_BLOCK(64, SPEC_BIG), ss>>>(SL);
                else if (L >= 16) seed_group_kernel<16, SPEC_MAX, false><<<sb((uint64_t)na * 16), 256, SEED_LDS_BLOCK(16, SPEC_MAX), ss>>>(SL);
                else if (L >= 4)  seed_group_kernel<4, SPEC_MAX, false><<<sb((uint64_t)na * 4), 256, SEED_LDS_BLOCK(4, SPEC_MAX), ss>>>(SL);
                else if (L >= 2)  seed_group_kernel<2, SPEC_MAX, false><<<sb((uint64_t)na * 2), 256, SEED_LDS_BLOCK(2, SPEC_MAX), ss>>>(SL);
                else              seed_kernel<false><<<sb(na), 256, 0, ss>>>(SL);
            }
            POISON_SYNC(ss, "seed kernel", c);
            HIPCHK(hipEventRecord(e1, ss));
            HIPCHK(hipGetLastError());
            return 0;
        };
        auto seed_time = [&](imsame_stats &sx, hipEvent_t e0, hipEvent_t e1, uint32_t na) -> int {
            float fs = 0;
            HIPCHK(hipEventElapsedTime(&fs, e0, e1));
            sx.ms_seed += fs;
            if (c->origin && timeline_on()) {
                float a = 0;
                if (hipEventElapsedTime(&a, c->origin, e0) == hipSuccess) {
                    std::lock_guard<std::mutex> g(c->iv_mu);
                    c->tl.push_back({'S', t_round, na, a, a + fs});
                }
            }
            return 0;
        };
        auto rec_launch = [&](imsame_stats &sx, const NwPlan &pl, uint32_t nc, double ms) {
            if (sx.nw_launches < IMSAME_LAUNCH_STATS) {
                sx.launch_cand[sx.nw_launches] = nc;
                sx.launch_ms[sx.nw_launches] = ms;
                if (pl.pk) sx.launch_pk |= 1ull << sx.nw_launches;
                if (pl.pk && pl.k == NW16_K5) sx.launch_k5 |= 1ull << sx.nw_launches;
                if (pl.pk && pl.k == NW16_K3) sx.launch_k3 |= 1ull << sx.nw_launches;
                if (pl.np) sx.launch_np |= 1ull << sx.nw_launches;
                if (pl.pk && pl.k == NW16_K19) sx.launch_k19 |= 1ull << sx.nw_launches;
                if (pl.lp) sx.launch_nwp |= 1ull << sx.nw_launches;
            }
            sx.ms_nw += ms; sx.nw_launches++; sx.n_nw += nc;
        };
        auto upd_launch = [&](const uint32_t *cr, const uint32_t *cs, uint32_t nc, const imsame_read_result *o,
                              uint32_t *next, int nnext_slot, hipStream_t ss, const uint32_t *uperm = nullptr) -> int {
            UpdLaunch U = {cr, cs, nc, o, read_from, c->res.as<imsame_read_result>(),
                           c->rstat.as<uint8_t>(), c->memo.as<uint32_t>(), c->nmemo.as<uint8_t>(),
                           c->cbase.as<uint32_t>(), c->ccnt.as<uint32_t>(), c->perr.as<uint32_t>(),
                           c->cur_p.as<uint64_t>(), next,
                           (uint32_t *)(ctr + nnext_slot), (unsigned long long *)(ctr + C_CELLS),
                           (unsigned long long *)(ctr + C_NACC), (unsigned long long *)(ctr + C_ERR),
                           c->db_start.as<uint64_t>(), ctr + C_FLAGS, (unsigned long long *)(ctr + C_WASTE), uperm};
            update_kernel<<<std::min<unsigned>(nblk(nc, 256), upd_blocks()), 256, 0, ss>>>(U);
            POISON_SYNC(ss, "update_kernel", c);
            HIPCHK(hipGetLastError());
            return 0;
        };
        // Split rounds (rounds >= 2 of many reads, short reads only).  A lane
        // alternates scan and NW round by round, and where every lane scans at
        // once the chip runs no NW (C3: ~39 ms of a 385 ms step,
        // profiles/r5zb/).  The round's active reads are scanned in two
        // halves, the second on stream_b, and each half's NW launch starts as
        // soon as its own scan is done: the first half's NW runs while the
        // second half scans.  The halves hold different reads, so each read
        // sees the same scan and the same NW results in the same order as in
        // one launch (tests).  IMSAME_SPLIT_ROUNDS=0 turns it off;
        // IMSAME_SPLIT_MIN sets the reads below which a round stays whole.
        if (RP.split(rnd, nact)) {
            if (!c->stream_b) {
                HIPCHK(hipStreamCreateWithFlags(&c->stream_b, hipStreamNonBlocking));
                HIPCHK(hipEventCreate(&c->evb0));
                HIPCHK(hipEventCreate(&c->evb1));
                for (int k = 0; k < 2; ++k)
                    HIPCHK(hipEventCreateWithFlags(&c->evw[1][k], hipEventBlockingSync | hipEventDisableTiming));
            }
            hipStream_t sb = c->stream_b;
            const char *sf = getenv("IMSAME_SPLIT_FRAC");            // the first half's share
            const double fa = sf ? std::max(0.05, std::min(0.95, atof(sf))) : 0.5;
            const uint32_t nA = std::max<uint32_t>(1, (uint32_t)(nact * fa)), nB = nact - nA;
            // the first half's list room: a read with no rejection yet may emit
            // up to spec_weak (spec_after_first), more than spec when IMSAME_SPEC
            // is set below it; nact x max(spec, spec_weak) <= ccap (RoundPolicy)
            const uint64_t offB = (uint64_t)std::max(S.spec, S.spec_weak) * nA;
            // stream_b starts behind what stream s has queued (the counters' reset)
            HIPCHK(hipEventRecord(c->evb0, s));
            HIPCHK(hipStreamWaitEvent(sb, c->evb0, 0));
            S.n_active = nA;
            SeedLaunch Sb = S;
            Sb.active = act + nA; Sb.n_active = nB;
            Sb.cread = c->cread.as<uint32_t>() + offB; Sb.csid = c->csid.as<uint32_t>() + offB;
            Sb.ncand = (uint32_t *)(ctr + C_NCANDB); Sb.ncand2 = (uint32_t *)(ctr + C_NCAND2B);
            Sb.crow = crow ? crow + offB : nullptr;
            Sb.dbg = nullptr;
            if ((rc = seed_launch(S, nA, s, c->ev0, c->ev1))) return rc;
            // the second half scans after the first (beside its NW launch): two
            // scans at once would end together and start both launches late
            // (IMSAME_SPLIT_SEQ=0: at once)
            const char *sq = getenv("IMSAME_SPLIT_SEQ");
            if (!(sq && !atoi(sq))) HIPCHK(hipStreamWaitEvent(sb, c->ev1, 0));
            if ((rc = seed_launch(Sb, nB, sb, c->evb0, c->evb1))) return rc;
            uint64_t ha[2], hb[2];
            HIPCHK(hipMemcpyAsync(ha, ctr + C_NCAND, 16, hipMemcpyDeviceToHost, s));
            LANE_SYNC(c, s);
            if ((rc = seed_time(st, c->ev0, c->ev1, nA))) return rc;
            if (ha[1]) return IMSAME_E_STATE;                         // short reads only: cannot happen
            const uint32_t na1 = (uint32_t)ha[0];
            NwPlan pla = {}, plb = {};
            double msa = 0, msb = 0;
            if (na1) {
                if ((rc = plan_nw(c, short_y, xcap, na1, p, c->q_len_mult, &pla, true, c->q_len_uni))) return rc;
                rc = launch_nw(c, pla, c->cread.as<uint32_t>(), c->csid.as<uint32_t>(), na1, c->cout.as<imsame_read_result>(),
                               p->igap, p->egap, p, ymax, xcap, (uint32_t *)(ctr + C_WORK), c->db.as<uint8_t>(),
                               c->db_start.as<uint64_t>(), qd, qsd, pcap, &msa, crow, 0, false);
                if (rc) return rc;
                if ((rc = upd_launch(c->cread.as<uint32_t>(), c->csid.as<uint32_t>(), na1, c->cout.as<imsame_read_result>(),
                                     nxt, C_NNEXT, s))) return rc;
            }
            HIPCHK(hipMemcpyAsync(hb, ctr + C_NCANDB, 16, hipMemcpyDeviceToHost, sb));
            LANE_SYNC(c, sb);
            if ((rc = seed_time(st, c->evb0, c->evb1, nB))) return rc;
            if (hb[1]) return IMSAME_E_STATE;
            const uint32_t nb1 = (uint32_t)hb[0];
            bool a_done = na1 == 0;
            if (nb1) {
                if ((rc = plan_nw(c, short_y, xcap, nb1, p, c->q_len_mult, &plb, true, c->q_len_uni))) return rc;
                // both launches share the arena only as non-persistent launches of one
                // slot layout; otherwise the second waits for the first (as round 1b)
                const bool same = pla.np && plb.np && plb.slot_words == pla.slot_words && plb.tb_dw == pla.tb_dw &&
                                  plb.ck_dw == pla.ck_dw && plb.bnd_dw == pla.bnd_dw && plb.max_blocks == pla.max_blocks;
                if (!same && !a_done) {
                    if ((rc = nw_launch_done(c, 0, na1, &msa))) return rc;
                    rec_launch(st, pla, na1, msa);
                    a_done = true;
                }
                rc = launch_nw(c, plb, Sb.cread, Sb.csid, nb1, c->cout.as<imsame_read_result>() + offB, p->igap, p->egap,
                               p, ymax, xcap, (uint32_t *)(ctr + C_WORKB), c->db.as<uint8_t>(), c->db_start.as<uint64_t>(),
                               qd, qsd, pcap, &msb, Sb.crow, 1, false);
                if (rc) return rc;
                if ((rc = upd_launch(Sb.cread, Sb.csid, nb1, c->cout.as<imsame_read_result>() + offB, nxt, C_NNEXT, sb)))
                    return rc;
            }
            if (!a_done) {
                if ((rc = nw_launch_done(c, 0, na1, &msa))) return rc;
                rec_launch(st, pla, na1, msa);
            }
            if (nb1) {
                if ((rc = nw_launch_done(c, 1, nb1, &msb))) return rc;
                rec_launch(st, plb, nb1, msb);
            }
            LANE_SYNC(c, sb);
            uint64_t nn = 0;
            HIPCHK(hipMemcpyAsync(&nn, ctr + C_NNEXT, 8, hipMemcpyDeviceToHost, s));
            LANE_SYNC(c, s);
            if (getenv("IMSAME_DEBUG_ROUNDS"))
                fprintf(stderr, "[round %llu split] active=%u+%u spec=%u budget=%u cand=%u+%u next=%llu\n",
                        (unsigned long long)st.rounds, nA, nB, S.spec, S.budget, na1, nb1, (unsigned long long)nn);
            if (na1 + nb1 == 0 && nn == 0) break;
            nact = (uint32_t)nn;
            std::swap(act, nxt);
            continue;
        }
        if ((rc = seed_launch(S, nact, s, c->ev0, c->ev1))) return rc;
        uint64_t hc[3];
        HIPCHK(hipMemcpyAsync(hc, ctr + C_NCAND, 24, hipMemcpyDeviceToHost, s));
        LANE_SYNC(c, s);
        if ((rc = seed_time(st, c->ev0, c->ev1, nact))) return rc;
        const uint32_t n1 = (uint32_t)hc[0], n2 = (uint32_t)hc[1];
        if (n1 + n2 + hc[2] == 0) break;                          // no candidates, nobody paused
        // Round 1b.  Reads that paused in round 1 without a candidate (budget
        // spent: at C2 the 10 % random reads, which scan every window) need
        // none of round 1's NW results, so their scan goes on at once on a
        // second stream, with speculation from a weak first pass, while the
        // round-1 NW launch runs; their candidates' NW launch joins it on
        // the chip.  Round 2 then holds the reads whose round-1 candidates
        // were rejected and the few the 1b scan paused (C2 shard 1/8: ~70 per
        // lane instead of ~6.3k, profiles/r3*).  Same visiting order per read,
        // so the same results (tests).  Short reads, both NW launches
        // non-persistent (they share the arena and its slot bitmap);
        // IMSAME_ROUND1B=0 turns it off.
        NwPlan pla = {};
        bool r1b = RP.r1b(rnd, n1, n2, hc[2]);
        if (r1b && n1 && (rc = plan_nw(c, short_y, xcap, n1, p, c->q_len_mult, &pla, true, c->q_len_uni))) return rc;
        if (r1b && n1 && !pla.np) r1b = false;
        // Independent pipelines (round 6).  The reads with round-1 candidates
        // (A) and the reads round 1 paused without one (B, round 1b's scan) are
        // disjoint and never need each other's NW results, so from round 1 on
        // each runs its own rounds to the end on its own stream -- A on the
        // lane's stream, B on stream_b from a host thread of its own -- with its
        // own active lists (A: act0 / act3, B: act1 / act2), counters (C_NCAND..
        // / C_NCANDB..) and part of the candidate lists (A: [0, n1), B: [n1,
        // ccap)).  Joined, both waited for the LATER of the two round-1 launches
        // before round 2: at C2 B's launch ends 20-30 ms before A's, and its
        // round-2 reads (most of round 2: random reads whose weak candidates
        // were rejected) sat behind A's (profiles/r6b/ timeline).  Same scans,
        // budgets and visiting order per read, so the same results (tests).
        // IMSAME_PIPES=0: the joined rounds below.
        if (r1b && pipes_on(n)) {
            if (!c->stream_b) {
                HIPCHK(hipStreamCreateWithFlags(&c->stream_b, hipStreamNonBlocking));
                HIPCHK(hipEventCreate(&c->evb0));
                HIPCHK(hipEventCreate(&c->evb1));
                for (int k = 0; k < 2; ++k)
                    HIPCHK(hipEventCreateWithFlags(&c->evw[1][k], hipEventBlockingSync | hipEventDisableTiming));
            }
            hipStream_t sb = c->stream_b;
            const uint32_t npz = (uint32_t)hc[2];
            uint32_t *cr0 = c->cread.as<uint32_t>(), *cs0 = c->csid.as<uint32_t>();
            imsame_read_result *co0 = c->cout.as<imsame_read_result>();
            // B's round 1b scan, as the joined form's
            SeedLaunch Sb = S;
            Sb.active = nxt; Sb.n_active = npz;
            Sb.spec = 1;
            Sb.spec_weak = RP.r1b_spec_weak(n1, npz);
            Sb.budget = RP.r1b_budget();
            Sb.next = c->act2.as<uint32_t>(); Sb.nnext = (uint32_t *)(ctr + C_NNEXT2);
            Sb.cread = cr0 + n1; Sb.csid = cs0 + n1;
            Sb.ncand = (uint32_t *)(ctr + C_NCANDB); Sb.crow = crow && RP.r1b_rows ? crow + n1 : nullptr;
            Sb.ncand2 = (uint32_t *)(ctr + C_NCAND2B);
            Sb.dbg = nullptr;
            if ((rc = seed_launch(Sb, npz, sb, c->evb0, c->evb1))) return rc;
            // a pipeline's state: stream (qi 0 / 1) and its events, lists,
            // candidate region [off, off + room), counter slots (cn: ncand,
            // ncand2, nnext; cw: its NW launch's work counter), round
            struct Pipe { hipStream_t s; int qi; hipEvent_t e0, e1; uint32_t *act, *nxt; uint32_t nact;
                          uint64_t off, room; int cn, cw; uint32_t rnd; };
            // one NW launch of a pipeline's candidates + its update (next list:
            // P.nxt, or `next` / counter slot `nslot`; perm: the candidates are
            // perm[0 .. nc) of the pipeline's part, whole reads' sets)
            auto pipe_nw = [&](Pipe &P, imsame_stats &sx, NwPlan &pl, uint32_t nc, const int32_t *cw_row,
                               const uint32_t *perm = nullptr, uint32_t *next = nullptr, int nslot = -1) -> int {
                // a launch that is not non-persistent uses this lane's own arena:
                // one at a time (launch_nw waits for it: wait = true)
                std::unique_lock<std::mutex> lk(c->persist_mu, std::defer_lock);
                if (!pl.np) lk.lock();
                double ms = 0;
                int r = launch_nw(c, pl, cr0 + P.off, cs0 + P.off, nc, co0 + P.off, p->igap, p->egap, p, ymax, xcap,
                                  (uint32_t *)(ctr + P.cw), c->db.as<uint8_t>(), c->db_start.as<uint64_t>(), qd, qsd,
                                  pcap, &ms, cw_row, P.qi, true, perm);
                if (r) return r;
                if (lk.owns_lock()) lk.unlock();
                rec_launch(sx, pl, nc, ms);
                return upd_launch(cr0 + P.off, cs0 + P.off, nc, co0 + P.off, next ? next : P.nxt,
                                  nslot >= 0 ? nslot : P.cn + 2, P.s, perm);
            };
            // rounds >= 2 of a pipeline, to its end
            auto pipe_rounds = [&](Pipe &P, imsame_stats &sx) -> int {
                while (P.nact) {
                    ++P.rnd;
                    t_round = (int)P.rnd;
                    HIPCHK(hipMemsetAsync(ctr + P.cn, 0, 3 * 8, P.s));       // ncand, ncand2, nnext
                    SeedLaunch Sp = S;
                    Sp.active = P.act; Sp.n_active = P.nact;
                    // speculation within this pipeline's part of the lists
                    const uint64_t room = std::max<uint64_t>(1, P.room / P.nact);
                    const uint64_t w = (!RP.spec_set && RP.pick_L(P.rnd, P.nact) >= 64) ? SPEC_BIG : RP.spec_later;
                    Sp.spec = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(w, room));
                    Sp.spec_weak = (uint32_t)std::min<uint64_t>(RP.spec_weak, room);
                    Sp.budget = RP.budget(P.rnd);
                    Sp.next = P.nxt; Sp.nnext = (uint32_t *)(ctr + P.cn + 2);
                    Sp.cread = cr0 + P.off; Sp.csid = cs0 + P.off;
                    Sp.ncand = (uint32_t *)(ctr + P.cn); Sp.ncand2 = (uint32_t *)(ctr + P.cn + 1);
                    Sp.crow = crow ? crow + P.off : nullptr;
                    Sp.dbg = nullptr;
                    if (int r = seed_launch(Sp, P.nact, P.s, P.e0, P.e1, P.rnd)) return r;
                    uint64_t hp[3];
                    HIPCHK(hipMemcpyAsync(hp, ctr + P.cn, 24, hipMemcpyDeviceToHost, P.s));
                    LANE_SYNC(c, P.s);
                    if (int r = seed_time(sx, P.e0, P.e1, P.nact)) return r;
                    if (hp[1]) return IMSAME_E_STATE;                   // short reads only: cannot happen
                    const uint32_t nc = (uint32_t)hp[0];
                    if (nc + hp[2] == 0) break;
                    if (nc) {
                        NwPlan pl;
                        if (int r = plan_nw(c, short_y, xcap, nc, p, c->q_len_mult, &pl, true, c->q_len_uni)) return r;
                        if (int r = pipe_nw(P, sx, pl, nc, crow ? crow + P.off : nullptr)) return r;
                    }
                    uint64_t nn = 0;
                    HIPCHK(hipMemcpyAsync(&nn, ctr + P.cn + 2, 8, hipMemcpyDeviceToHost, P.s));
                    LANE_SYNC(c, P.s);
                    if (getenv("IMSAME_DEBUG_ROUNDS"))
                        fprintf(stderr, "[round %u pipe %c] active=%u spec=%u budget=%u cand=%u next=%llu\n", P.rnd,
                                P.qi ? 'B' : 'A', P.nact, Sp.spec, Sp.budget, nc, (unsigned long long)nn);
                    P.nact = (uint32_t)nn;
                    std::swap(P.act, P.nxt);
                }
                return 0;
            };
            // B, on its own host thread: round 1's unpredicted candidates' and
            // round 1b's NW launches + updates, then its rounds
            imsame_stats stB;
            memset(&stB, 0, sizeof stB);
            // Round 1's launch is cut in two by the row order (row_perm): the
            // UNPREDICTED candidates (weak first hits: random reads, whose
            // candidates are all unpredicted; the front of the order) run on
            // B's stream after the 1b scan and their update appends the rejected
            // reads to B's list; the PREDICTED ones (true reads, one candidate
            // each) run on A's stream at once, A's list.  Most later-round reads
            // are the weak ones (C2: ~6.4k of a lane's ~6.5k round-2 reads,
            // profiles/r6c/), so round 2 now scans on beside the true reads'
            // launch instead of after it.  (Run first on A's stream, the weak
            // launch and its update delayed the true reads' launch by 5-17 ms
            // at C2: profiles/r6d/.)  A hands B the cut through wstate: 1 with
            // nw / pm set (ev_w after the perm on A's stream), -1 if A failed.
            std::mutex wmu;
            std::condition_variable wcv;
            int wstate = 0;
            uint32_t nw = 0;
            const uint32_t *pm = nullptr;
            auto w_done = [&](int v) { { std::lock_guard<std::mutex> g(wmu); wstate = v; } wcv.notify_all(); };
            // ... and B hands A the end of the weak launch back through wdstate
            // (1: ev_wd recorded after its update, -1: B failed): the weak launch
            // and its update read the cut (pm = A's cperm), which A's next
            // launches rewrite with their own row order
            int wdstate = 0;
            auto wd_done = [&](int v) { { std::lock_guard<std::mutex> g(wmu); wdstate = v; } wcv.notify_all(); };
            if (!c->ev_w) HIPCHK(hipEventCreateWithFlags(&c->ev_w, hipEventDisableTiming));
            if (!c->ev_wd) HIPCHK(hipEventCreateWithFlags(&c->ev_wd, hipEventDisableTiming));
            // (B.act: round 1b's active list, act1; its update appends to B.nxt,
            // act2, where the 1b scan put the reads it paused -- round 2's list)
            Pipe B = {sb, 1, c->evb0, c->evb1, nxt, c->act2.as<uint32_t>(), 0, n1, ccap - n1, C_NCANDB, C_WORKB, 1};
            int rcB = 0;
            std::thread thB([&] {
                rcB = [&]() -> int {
                    HIPCHK(hipSetDevice(c->device));
                    t_round = 1;
                    uint64_t hb[2];
                    HIPCHK(hipMemcpyAsync(hb, ctr + C_NCANDB, 16, hipMemcpyDeviceToHost, sb));
                    LANE_SYNC(c, sb);                    // the 1b scan (its events: before a launch reuses them)
                    if (int r = seed_time(stB, c->evb0, c->evb1, npz)) return r;
                    {
                        std::unique_lock<std::mutex> g(wmu);
                        wcv.wait(g, [&] { return wstate != 0; });
                        if (wstate < 0) return IMSAME_E_STATE;   // A failed before it: A reports it
                    }
                    if (nw) {                            // the unpredicted candidates (A's part of the lists)
                        HIPCHK(hipStreamWaitEvent(sb, c->ev_w, 0));
                        Pipe W = B;
                        W.off = 0; W.room = n1;
                        NwPlan plw;
                        if (int r = plan_nw(c, short_y, xcap, nw, p, c->q_len_mult, &plw, true, c->q_len_uni)) return r;
                        if (int r = pipe_nw(W, stB, plw, nw, crow, pm, c->act2.as<uint32_t>(), C_NNEXT2)) return r;
                        HIPCHK(hipEventRecord(c->ev_wd, sb));
                    }
                    wd_done(1);
                    if (hb[1]) return IMSAME_E_STATE;
                    const uint32_t nb = (uint32_t)hb[0];
                    if (nb) {
                        NwPlan plb;
                        if (int r = plan_nw(c, short_y, xcap, nb, p, c->q_len_mult, &plb, true, c->q_len_uni)) return r;
                        if (int r = pipe_nw(B, stB, plb, nb, Sb.crow)) return r;
                    }
                    uint64_t nn = 0;
                    HIPCHK(hipMemcpyAsync(&nn, ctr + C_NNEXT2, 8, hipMemcpyDeviceToHost, sb));
                    LANE_SYNC(c, sb);
                    B.nact = (uint32_t)nn;
                    std::swap(B.act, B.nxt);             // round 2 scans act2; act1 is free
                    return pipe_rounds(B, stB);
                }();
                if (!wdstate) wd_done(-1);               // (B failed before the weak launch ended)
            });
            // A, on this thread: the cut, round 1's predicted candidates' launch
            // + update (its next list: act3; C_NNEXT held round 1's paused
            // count), then its rounds
            Pipe A = {s, 0, c->ev0, c->ev1, c->act3.as<uint32_t>(), act, 0, 0, n1, C_NCAND, C_WORK, 1};
            const int rcA = [&]() -> int {
                HIPCHK(hipMemsetAsync(ctr + C_NNEXT, 0, 8, s));
                if (n1 && crow && pla.two && cut_weak_on()) {
                    uint32_t k = 0;
                    if (int r = row_perm(c, crow, n1, (uint32_t)pla.xcap, 0, &k)) return r;
                    nw = k; pm = c->cperm.as<uint32_t>();
                    HIPCHK(hipEventRecord(c->ev_w, s));
                }
                w_done(1);
                if (getenv("IMSAME_DEBUG_ROUNDS"))
                    fprintf(stderr, "[round 1 pipes] cand=%u unpredicted=%u paused=%u\n", n1, nw, npz);
                if (n1 > nw) {                           // the predicted ones
                    NwPlan pls = pla;
                    if (nw && (rc = plan_nw(c, short_y, xcap, n1 - nw, p, c->q_len_mult, &pls, true, c->q_len_uni)))
                        return rc;
                    std::swap(A.act, A.nxt);             // the update writes A.nxt = act3
                    const int r = pipe_nw(A, st, pls, n1 - nw, crow, pm ? pm + nw : nullptr);
                    std::swap(A.act, A.nxt);
                    if (r) return r;
                }
                uint64_t nn = 0;
                HIPCHK(hipMemcpyAsync(&nn, ctr + C_NNEXT, 8, hipMemcpyDeviceToHost, s));
                LANE_SYNC(c, s);
                A.nact = (uint32_t)nn;
                if (nw && A.nact) {                      // A's next launches rewrite cperm
                    std::unique_lock<std::mutex> g(wmu);
                    wcv.wait(g, [&] { return wdstate != 0; });
                    if (wdstate < 0) return IMSAME_E_STATE;   // B failed: B reports it
                    HIPCHK(hipStreamWaitEvent(s, c->ev_wd, 0));
                }
                return pipe_rounds(A, st);
            }();
            if (!wstate) w_done(-1);                     // (A failed before its first launch)
            thB.join();
            if (rcA) return rcA;
            if (rcB) return rcB;
            c->b_prio = stB.n_nw > st.n_nw;             // for the next call (prio_b)
            // one stats record: B's launches after A's
            st.rounds = std::max(A.rnd, B.rnd);
            st.ms_seed += stB.ms_seed;
            for (uint64_t j = 0; j < std::min<uint64_t>(stB.nw_launches, IMSAME_LAUNCH_STATS); ++j) {
                const uint64_t d = st.nw_launches + j;
                if (d >= IMSAME_LAUNCH_STATS) break;
                st.launch_cand[d] = stB.launch_cand[j]; st.launch_ms[d] = stB.launch_ms[j];
                const uint64_t bit = 1ull << j, to = 1ull << d;
                if (stB.launch_pk & bit) st.launch_pk |= to;
                if (stB.launch_k5 & bit) st.launch_k5 |= to;
                if (stB.launch_k3 & bit) st.launch_k3 |= to;
                if (stB.launch_np & bit) st.launch_np |= to;
                if (stB.launch_k19 & bit) st.launch_k19 |= to;
                if (stB.launch_nwp & bit) st.launch_nwp |= to;
            }
            st.ms_nw += stB.ms_nw; st.nw_launches += stB.nw_launches; st.n_nw += stB.n_nw;
            break;
        }
        if (r1b) {
            if (!c->stream_b) {
                HIPCHK(hipStreamCreateWithFlags(&c->stream_b, hipStreamNonBlocking));
                HIPCHK(hipEventCreate(&c->evb0));
                HIPCHK(hipEventCreate(&c->evb1));
                for (int k = 0; k < 2; ++k)
                    HIPCHK(hipEventCreateWithFlags(&c->evw[1][k], hipEventBlockingSync | hipEventDisableTiming));
            }
            hipStream_t sb = c->stream_b;
            uint32_t *act2 = c->act2.as<uint32_t>();
            const uint32_t npz = (uint32_t)hc[2];
            SeedLaunch Sb = S;
            Sb.active = nxt; Sb.n_active = npz;
            Sb.spec = 1;
            Sb.spec_weak = RP.r1b_spec_weak(n1, npz);
            Sb.budget = RP.r1b_budget();
            Sb.next = act2; Sb.nnext = (uint32_t *)(ctr + C_NNEXT2);
            Sb.cread = c->cread.as<uint32_t>() + n1; Sb.csid = c->csid.as<uint32_t>() + n1;
            Sb.ncand = (uint32_t *)(ctr + C_NCANDB); Sb.crow = crow && RP.r1b_rows ? crow + n1 : nullptr;
            Sb.ncand2 = (uint32_t *)(ctr + C_NCAND2B);
            Sb.dbg = nullptr;
            if ((rc = seed_launch(Sb, npz, sb, c->evb0, c->evb1))) return rc;
            double msa = 0, msb = 0;
            if (n1) {
                rc = launch_nw(c, pla, c->cread.as<uint32_t>(), c->csid.as<uint32_t>(), n1, c->cout.as<imsame_read_result>(),
                               p->igap, p->egap, p, ymax, xcap, (uint32_t *)(ctr + C_WORK), c->db.as<uint8_t>(),
                               c->db_start.as<uint64_t>(), qd, qsd, pcap, &msa, crow, 0, false);
                if (rc) return rc;
                if ((rc = upd_launch(c->cread.as<uint32_t>(), c->csid.as<uint32_t>(), n1, c->cout.as<imsame_read_result>(),
                                     act2, C_NNEXT2, s))) return rc;
            }
            uint64_t hb[2];
            HIPCHK(hipMemcpyAsync(hb, ctr + C_NCANDB, 16, hipMemcpyDeviceToHost, sb));
            LANE_SYNC(c, sb);                         // the 1b scan only: N1a runs on
            if ((rc = seed_time(st, c->evb0, c->evb1, npz))) return rc;
            const uint32_t nb = (uint32_t)hb[0];
            if (hb[1]) return IMSAME_E_STATE;                         // short reads only: cannot happen
            NwPlan plb = {};
            bool a_done = n1 == 0;
            if (nb) {
                if ((rc = plan_nw(c, short_y, xcap, nb, p, c->q_len_mult, &plb, true, c->q_len_uni))) return rc;
                // N1a's launch_nw may have fallen back to a persistent launch on
                // this lane's own arena: then N1b must wait for it (pla.np is
                // what it ran with)
                const bool same = pla.np && plb.np && plb.slot_words == pla.slot_words && plb.tb_dw == pla.tb_dw &&
                                  plb.ck_dw == pla.ck_dw && plb.bnd_dw == pla.bnd_dw && plb.max_blocks == pla.max_blocks;
                if (!same && !a_done) {                               // not N1a's arena layout: after it
                    if ((rc = nw_launch_done(c, 0, n1, &msa))) return rc;
                    rec_launch(st, pla, n1, msa);
                    a_done = true;
                }
                rc = launch_nw(c, plb, c->cread.as<uint32_t>() + n1, c->csid.as<uint32_t>() + n1, nb,
                               c->cout.as<imsame_read_result>() + n1, p->igap, p->egap, p, ymax, xcap,
                               (uint32_t *)(ctr + C_WORKB), c->db.as<uint8_t>(), c->db_start.as<uint64_t>(), qd, qsd,
                               pcap, &msb, Sb.crow, 1, false);
                if (rc) return rc;
                if ((rc = upd_launch(c->cread.as<uint32_t>() + n1, c->csid.as<uint32_t>() + n1, nb,
                                     c->cout.as<imsame_read_result>() + n1, act2, C_NNEXT2, sb))) return rc;
            }
            if (!a_done) {
                if ((rc = nw_launch_done(c, 0, n1, &msa))) return rc;
                rec_launch(st, pla, n1, msa);
            }
            if (nb) {
                if ((rc = nw_launch_done(c, 1, nb, &msb))) return rc;
                rec_launch(st, plb, nb, msb);
            }
            LANE_SYNC(c, sb);
            uint64_t nn = 0;
            HIPCHK(hipMemcpyAsync(&nn, ctr + C_NNEXT2, 8, hipMemcpyDeviceToHost, s));
            LANE_SYNC(c, s);
            if (getenv("IMSAME_DEBUG_ROUNDS"))
                fprintf(stderr, "[round 1b] paused=%u spec_weak=%u budget=%u cand=%u+%u next=%llu | a: k%d np%d sw%u tb%llu ck%llu "
                        "mb%u | b: k%d np%d sw%u tb%llu ck%llu mb%u\n", npz, Sb.spec_weak, Sb.budget, n1, nb,
                        (unsigned long long)nn, pla.k, (int)pla.np, pla.slot_words, (unsigned long long)pla.tb_dw,
                        (unsigned long long)pla.ck_dw, pla.max_blocks, nb ? plb.k : -1, nb ? (int)plb.np : -1,
                        nb ? plb.slot_words : 0u, nb ? (unsigned long long)plb.tb_dw : 0ull,
                        nb ? (unsigned long long)plb.ck_dw : 0ull, nb ? plb.max_blocks : 0u);
            nact = (uint32_t)nn;
            nxt = act; act = act2;                                    // round 2 scans act2; act0 is free
            continue;
        }
        struct Cls { uint32_t n; uint32_t *cr, *cs; imsame_read_result *o; uint32_t ylim; int work; };
        Cls cls[2] = {{n1, c->cread.as<uint32_t>(), c->csid.as<uint32_t>(), c->cout.as<imsame_read_result>(), short_y, C_WORK},
                      {n2, c->cread2.as<uint32_t>(), c->csid2.as<uint32_t>(), c->cout2.as<imsame_read_result>(), ycap, C_WORK2}};
        for (int k = 0; k < 2; ++k) {
            if (!cls[k].n) continue;
            NwPlan pl;
            if ((rc = plan_nw(c, cls[k].ylim, xcap, cls[k].n, p, c->q_len_mult, &pl, true, c->q_len_uni))) return rc;
            double ms = 0;
            rc = launch_nw(c, pl, cls[k].cr, cls[k].cs, cls[k].n, cls[k].o, p->igap, p->egap, p, ymax, xcap,
                           (uint32_t *)(ctr + cls[k].work), c->db.as<uint8_t>(), c->db_start.as<uint64_t>(), qd, qsd,
                           pcap, &ms, k == 0 ? crow : nullptr);
            if (rc) return rc;
            rec_launch(st, pl, cls[k].n, ms);
            if ((rc = upd_launch(cls[k].cr, cls[k].cs, cls[k].n, cls[k].o, nxt, C_NNEXT, s))) return rc;
        }
        uint64_t nn = 0;
        HIPCHK(hipMemcpyAsync(&nn, ctr + C_NNEXT, 8, hipMemcpyDeviceToHost, s));
        LANE_SYNC(c, s);
        if (getenv("IMSAME_DEBUG_ROUNDS")) {      // diagnostics: per-round shape + a few candidates
            std::vector<imsame_read_result> o(std::min<uint32_t>(n1, 6));
            std::vector<uint32_t> cr(o.size());
            if (!o.empty()) {
                HIPCHK(hipMemcpy(o.data(), c->cout.p, o.size() * 64, hipMemcpyDeviceToHost));
                HIPCHK(hipMemcpy(cr.data(), c->cread.p, o.size() * 4, hipMemcpyDeviceToHost));
            }
            uint64_t dg[8], nacc = 0;
            HIPCHK(hipMemcpy(dg, ctr + C_DBG, sizeof dg, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(&nacc, ctr + C_NACC, 8, hipMemcpyDeviceToHost));
            fprintf(stderr, "[round %llu] active=%u spec=%u budget=%u cand=%u+%u next=%llu acc_total=%llu "
                    "outcomes(err0 pause0 done0 err pause exh full)=%llu %llu %llu %llu %llu %llu %llu |",
                    (unsigned long long)st.rounds, nact, S.spec, S.budget, n1, n2, (unsigned long long)nn,
                    (unsigned long long)nacc, (unsigned long long)dg[0], (unsigned long long)dg[1],
                    (unsigned long long)dg[2], (unsigned long long)dg[3], (unsigned long long)dg[4],
                    (unsigned long long)dg[5], (unsigned long long)dg[6]);
            for (size_t k = 0; k < o.size(); ++k)
                fprintf(stderr, " r%u/s%llu st%u len%u id%u y%u", cr[k], (unsigned long long)o[k].db_seq, o[k].status,
                        o[k].length, o[k].identities, o[k].ylen);
            fprintf(stderr, "\n");
        }
        nact = (uint32_t)nn;
        std::swap(act, nxt);
    }
    uint64_t hc[C_NSLOTS];
    HIPCHK(hipMemcpyAsync(hc, ctr, C_NSLOTS * 8, hipMemcpyDeviceToHost, s));
    LANE_SYNC(c, s);
    const double t_d2h = now_ms();
    HIPCHK(hipMemcpyAsync(res, c->res.p, (uint64_t)n * 64, hipMemcpyDeviceToHost, s));
    LANE_SYNC(c, s);
    st.ms_d2h = now_ms() - t_d2h;
    st.n_hits = hc[C_HITS];
    st.seed_windows = hc[C_SWORK]; st.seed_entries = hc[C_SWORK + 1]; st.seed_ext_chunks = hc[C_SWORK + 2];
    st.nw_cells = hc[C_CELLS];
    st.n_accepted = hc[C_NACC];
    st.nw_redo = (uint32_t)hc[C_REDO];
    st.nw_win = (uint32_t)hc[C_WIN];
    st.nw_fallback = (uint32_t)hc[C_FBK];
    st.nw_spec_waste = hc[C_WASTE];
    if (getenv("IMSAME_NW_PROF")) {           // diagnostics: nw16 phase cycles (summed over waves)
        const double tot = (double)(hc[C_PROF] + hc[C_PROF + 1] + hc[C_PROF + 2] + hc[C_PROF + 3] + hc[C_PROF + 4]);
        // shader clock under this load: the waves' cycles over their 100 MHz real time
        const double ghz = hc[C_PROF + 5] ? tot / (double)hc[C_PROF + 5] * 0.1 : 0.0;
        fprintf(stderr, "[nwprof] setup %.3f sweep1 %.3f reduce %.3f sweep2 %.3f walk %.3f (fractions of %.4g wave-cycles) "
                "clock_ghz %.3f best_cells(weak: last_row last_col<=40 <=200 higher | predicted: in out) "
                "%llu %llu %llu %llu | %llu %llu\n", hc[C_PROF] / tot, hc[C_PROF + 1] / tot, hc[C_PROF + 2] / tot,
                hc[C_PROF + 3] / tot, hc[C_PROF + 4] / tot, tot, ghz, (unsigned long long)hc[C_PROF + 6],
                (unsigned long long)hc[C_PROF + 7], (unsigned long long)hc[C_PROF + 8], (unsigned long long)hc[C_PROF + 9],
                (unsigned long long)hc[C_PROF + 10], (unsigned long long)hc[C_PROF + 11]);
    }
    st.nw_launch_ms = st.nw_launches ? st.ms_nw / st.nw_launches : 0;
    st.nw_bytes = 2 * st.nw_cells;       // 2 B/cell traceback floor; bench.py adds xlen + ylen per NW
    int ret = IMSAME_OK;
    if (hc[C_FLAGS] & 4) return IMSAME_E_HIP;     // a non-persistent NW wave found no arena slot (never)
    if (hc[C_FLAGS] & 8) return IMSAME_E_ARG;     // a query byte that is not ACGT (pack2_kernel)
    if (hc[C_ERR] != ~0ull) {
        st.err_read = hc[C_ERR] >> 32; st.err_dbseq = hc[C_ERR] & 0xFFFFFFFFull;
        ret = IMSAME_E_READ_TOO_LONG;
    }
    if (p->want_paths) {
        uint64_t used = std::min<uint64_t>((uint32_t)hc[C_PATHS], pcap);
        if (hc[C_FLAGS] & 1) {
            rc = rewalk_lost(c, p, read_from, n, res, ymax, xcap, ycap, short_y, &used, &st);
            if (rc) return rc;
        }
        c->paths_n = used;
        c->paths_hint = std::min(64.0, (double)used / n);
        if (paths_used) *paths_used = used;
        if (used > paths_cap) { if (ret == IMSAME_OK) ret = IMSAME_E_PATHS; }
        else if (used) {
            HIPCHK(hipMemcpyAsync(paths, c->paths.p, used * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        }
    }
    st.ms_total = now_ms() - t_start;
    if (stats) *stats = st;
    return ret;
}

// first start and last end of [a, b) intervals (ms on the call's clock)
static void span_ms(const std::vector<std::pair<float, float>> &v, double *first, double *last) {
    *first = *last = 0;
    for (size_t k = 0; k < v.size(); ++k) {
        if (k == 0 || v[k].first < *first) *first = v[k].first;
        if (k == 0 || v[k].second > *last) *last = v[k].second;
    }
}

// total length of the union of [a, b) intervals
static double union_ms(std::vector<std::pair<float, float>> v) {
    std::sort(v.begin(), v.end());
    double tot = 0, a = 0, b = -1;
    for (const auto &x : v) {
        if (x.first > b) { if (b > a) tot += b - a; a = x.first; b = x.second; }
        else b = std::max<double>(b, x.second);
    }
    if (b > a) tot += b - a;
    return tot;
}

// Reads per lane below which a call is not split (a lane must fill the chip)
#define LANE_MIN 32768
#define LANE_READS 40000

// Hand lane l's finished reads [a, b) to an imsame_dev_align_parts callback,
// with its paths copied to the host (path_off of those rows index them).
static int deliver_part(imsame_ctx *l, const imsame_params *p, uint64_t a, uint64_t b, int rc, uint64_t used,
                        uint64_t err_read, imsame_part_fn fn, void *user) {
    const int status = (rc == IMSAME_E_PATHS) ? IMSAME_OK : rc;
    uint64_t np = 0;
    if (p->want_paths && used && (status == IMSAME_OK || status == IMSAME_E_READ_TOO_LONG)) {
        l->part_paths.resize(used);
        HIPCHK(hipMemcpyAsync(l->part_paths.data(), l->paths.p, used * 4, hipMemcpyDeviceToHost, l->stream));
        HIPCHK(hipStreamSynchronize(l->stream));
        np = used;
    }
    fn(user, a, b, status, status == IMSAME_E_READ_TOO_LONG ? err_read : ~0ull, np ? l->part_paths.data() : nullptr, np);
    return 0;
}

static int align_impl(imsame_ctx *c, uint64_t read_from, uint64_t read_to, uint64_t n_threads_semantic,
                      const imsame_params *p, imsame_read_result *res, uint32_t *paths, uint64_t paths_cap,
                      uint64_t *paths_used, imsame_stats *stats, imsame_part_fn fn, void *user);

extern "C" int imsame_dev_align(imsame_ctx *c, uint64_t read_from, uint64_t read_to, uint64_t n_threads_semantic,
                                const imsame_params *p, imsame_read_result *res, uint32_t *paths, uint64_t paths_cap,
                                uint64_t *paths_used, imsame_stats *stats) {
    return align_impl(c, read_from, read_to, n_threads_semantic, p, res, paths, paths_cap, paths_used, stats, nullptr,
                      nullptr);
}

extern "C" int imsame_dev_align_parts(imsame_ctx *c, uint64_t read_from, uint64_t read_to, uint64_t n_threads_semantic,
                                      const imsame_params *p, imsame_read_result *res, imsame_part_fn fn, void *user,
                                      imsame_stats *stats) {
    if (!fn) return IMSAME_E_ARG;
    uint64_t used = 0;
    return align_impl(c, read_from, read_to, n_threads_semantic, p, res, nullptr, 0, &used, stats, fn, user);
}

static int align_impl(imsame_ctx *c, uint64_t read_from, uint64_t read_to, uint64_t n_threads_semantic,
                      const imsame_params *p, imsame_read_result *res, uint32_t *paths, uint64_t paths_cap,
                      uint64_t *paths_used, imsame_stats *stats, imsame_part_fn fn, void *user) {
    const double t_start = now_ms();
    if (!c || !p || (!res && read_to > read_from)) return IMSAME_E_ARG;
    if (!c->have_index || !c->have_query) return IMSAME_E_STATE;
    if (read_from < c->q_lo || read_to > c->q_hi || read_from > read_to) return IMSAME_E_ARG;
    if (p->want_paths && !paths && paths_cap) return IMSAME_E_ARG;
    HIPCHK(hipSetDevice(c->device));
    if (!c->origin) HIPCHK(hipEventCreate(&c->origin));
    HIPCHK(hipEventRecord(c->origin, c->stream));          // common clock of every lane's NW launches
    c->nw_iv.clear();
    c->paths_split = false;
    const uint64_t n = read_to - read_from;
    uint64_t ymax = 0;
    ymax = range_ymax(c, read_from, read_to);
    if (!c->is_sub && ymax <= (uint64_t)NW_W / 2 && n) {   // the lanes' shared NW arena, before they start
        const int rp = np_prepare(c, (uint32_t)std::min<uint64_t>(c->max_rec, p->max_read_size));
        if (rp) return rp;
    }
    // LANES: the range is cut into `nl` parts that run concurrently on nl
    // streams (this context and c->subs, which share the index and the
    // query), so one part's latency-bound phases -- seed scans, the last
    // small NW launches, host round trips -- overlap the others' VALU-bound
    // NW sweeps.  Per-read results do not depend on the cut (reads are
    // independent given the chunk heads).  Short reads only: a long-read
    // lane's traceback arena takes most of HBM.
    // How many: from the work and the hardware queues.  A lane needs
    // LANE_READS reads for its first NW launch to fill the chip's wave slots
    // on its own (~0.9 candidates per read, 8 per wave: 40k reads -> 4.5k
    // waves against 4 per SIMD x 1024 SIMDs), and a hardware queue of its own
    // (lanes_for_queues), and at most LANES_DEF: with the 19-column NW form
    // and round 1b, 3 lanes are as fast as 4 on 1M reads (108.08 vs 108.05
    // ms) and on the 1/8 shard, faster on the 1/2 shard (58.0 vs 58.4 ms) and
    // on the 1/4 shard (31.7 vs 34.4-34.7 ms), and 8 lanes are slower
    // (profiles/r4i/, r4j/).  IMSAME_LANES overrides (tests, A/B runs).
    const char *le = getenv("IMSAME_LANES");
    const char *lre = getenv("IMSAME_LANE_READS");
    const uint64_t lane_reads = std::max<uint64_t>(1, lre ? strtoull(lre, nullptr, 10) : LANE_READS);
    int nl = le ? std::max(1, std::min(LANES_MAX, atoi(le)))
                : (int)std::max<uint64_t>(1, std::min<uint64_t>(std::min(std::min(lanes_for_queues(), LANES_DEF),
                                                                          host_threads_cap()), n / lane_reads));
    const char *lme = getenv("IMSAME_LANE_MIN");
    const uint64_t lane_min = lme ? strtoull(lme, nullptr, 10) : LANE_MIN;
    while (nl > 1 && n < (uint64_t)nl * lane_min) --nl;
    if (c->is_sub || c->use_wcap || ymax > (uint64_t)NW_W / 2) nl = 1;
    if (nl == 1) {
        imsame_stats s1{};
        int rc = align_one(c, read_from, read_to, n_threads_semantic, p, res, paths, paths_cap, paths_used, &s1);
        s1.ms_nw_busy = union_ms(c->nw_iv);
        span_ms(c->nw_iv, &s1.ms_nw_first, &s1.ms_nw_last);
        if (timeline_on()) timeline_print({c});
        if (stats) *stats = s1;
        if (fn) {
            const int rd = deliver_part(c, p, read_from, read_to, rc, paths_used ? *paths_used : 0, s1.err_read, fn, user);
            if (rd) return rd;
            if (rc == IMSAME_E_PATHS) rc = IMSAME_OK;
        }
        return rc;
    }
    std::vector<imsame_ctx *> L(nl, c);
    for (int k = 1; k < nl; ++k) {
        int rc = lane_sub(c, k, &L[k]);
        if (rc) return rc;
        L[k]->origin = c->origin;
        L[k]->nw_iv.clear();
    }
    for (int k = 0; k < nl; ++k) L[k]->nlanes = nl;


    // PIECES (callback calls only): each lane's share is cut into `ns`
    // pieces, piece i on lane i % nl, so the first nl pieces -- a prefix of
    // the range -- are handed over while the lanes align the rest, and the
    // caller's output of that prefix overlaps the device.  3 pieces: the CLI
    // at C2 writes its 3 GB with a render tail of 0.125-0.132 s instead of
    // 0.18-0.19 s, the alignment 0.122-0.123 -> 0.132-0.135 s, process wall
    // 0.70-0.77 -> 0.70-0.72 s (2 pieces: tail 0.140 s; profiles/r4p/, r4q/).
    // IMSAME_LANE_PARTS overrides (1: one piece per lane).
    const char *lpe = getenv("IMSAME_LANE_PARTS");
    int ns = !fn ? 1 : lpe ? std::max(1, std::min(16, atoi(lpe))) : 3;
    while (ns > 1 && n < (uint64_t)(nl * ns) * lane_min) --ns;
    const int np = nl * ns;
    std::vector<uint64_t> cut(np + 1), used(np, 0);
    // lane k's share grows linearly, weight 1 + x (2k/(nl-1) - 1): equal lanes
    // reach their latency-bound phases (update, next seed scan) at the same
    // moment and leave the chip idle together; x = 0.4 for 8 lanes (C2: +0.7 %
    // over four alternating pairs, profiles/r2ap_*, r2aq_*), IMSAME_LANE_SKEW
    const char *ske = getenv("IMSAME_LANE_SKEW");
    const double skew = ske ? std::max(-0.9, std::min(0.9, atof(ske))) : (nl >= 8 ? 0.4 : 0.0);
    {
        std::vector<double> w(np), acc(np + 1, 0.0);
        for (int i = 0; i < np; ++i) w[i] = 1.0 + skew * (nl > 1 ? 2.0 * (i % nl) / (nl - 1) - 1.0 : 0.0);
        for (int i = 0; i < np; ++i) acc[i + 1] = acc[i] + w[i];
        for (int i = 0; i <= np; ++i) cut[i] = read_from + (uint64_t)((double)n * acc[i] / acc[np]);
        cut[0] = read_from; cut[np] = read_to;
    }
    std::vector<imsame_stats> S(np);
    std::vector<int> R(np, 0);
    std::vector<std::thread> th;
    // each lane runs on its own host thread (lane 0 on the caller's) and,
    // with a callback, hands over each piece as soon as its reads are final;
    // a hard error ends the lane (the caller stops on it)
    auto lane_run = [&](int k) {
        for (int i = k; i < np; i += nl) {
            R[i] = align_one(L[k], cut[i], cut[i + 1], n_threads_semantic, p, res + (cut[i] - read_from), nullptr, 0,
                             &used[i], &S[i]);
            if (fn) {
                const int rd = deliver_part(L[k], p, cut[i], cut[i + 1], R[i], used[i], S[i].err_read, fn, user);
                if (rd) R[i] = rd;
            }
            if (R[i] && R[i] != IMSAME_E_PATHS && R[i] != IMSAME_E_READ_TOO_LONG) break;
        }
    };
    for (int k = 1; k < nl; ++k) th.emplace_back(lane_run, k);
    lane_run(0);
    for (auto &t : th) t.join();
    if (timeline_on()) timeline_print(L);
    for (int k = 1; k < nl; ++k) L[k]->origin = nullptr;
    for (int k = 0; k < nl; ++k) L[k]->nlanes = 1;
    for (int r : R)
        if (r && r != IMSAME_E_PATHS && r != IMSAME_E_READ_TOO_LONG) return r;
    int ret = IMSAME_OK;
    for (int r : R)
        if (r == IMSAME_E_READ_TOO_LONG) ret = IMSAME_E_READ_TOO_LONG;
    // one result set: each lane's paths follow the previous lanes' (parts:
    // each part's rows index its own paths, handed over in the callback;
    // without a callback a lane runs one piece, np == nl)
    uint64_t base = 0;
    for (int k = 0; k < np; ++k) {
        if (p->want_paths && k && !fn)
            for (uint64_t r = cut[k]; r < cut[k + 1]; ++r) {
                imsame_read_result &x = res[r - read_from];
                if (x.status == 1 && x.path_len) x.path_off += (uint32_t)base;
            }
        base += used[k];
    }
    imsame_stats st = S[0];
    std::vector<std::pair<float, float>> iv = c->nw_iv;
    for (int k = 1; k < nl; ++k) iv.insert(iv.end(), L[k]->nw_iv.begin(), L[k]->nw_iv.end());
    st.nw_launches = 0; st.launch_pk = 0; st.launch_k5 = 0; st.launch_np = 0; st.launch_k19 = 0; st.launch_nwp = 0;
    st.launch_k3 = 0;
    for (int k = 0; k < np; ++k) {
        const imsame_stats &x = S[k];
        if (k) {
            st.n_reads += x.n_reads; st.n_accepted += x.n_accepted; st.n_nw += x.n_nw; st.nw_cells += x.nw_cells;
            st.n_hits += x.n_hits; st.rounds = std::max(st.rounds, x.rounds);
            if (x.err_read < st.err_read) { st.err_read = x.err_read; st.err_dbseq = x.err_dbseq; }
            st.ms_seed += x.ms_seed; st.ms_nw += x.ms_nw; st.nw_bytes += x.nw_bytes; st.n_rewalk += x.n_rewalk;
            st.nw_redo += x.nw_redo; st.nw_win += x.nw_win; st.nw_fallback += x.nw_fallback;
            st.seed_windows += x.seed_windows; st.seed_entries += x.seed_entries;
            st.seed_ext_chunks += x.seed_ext_chunks; st.nw_spec_waste += x.nw_spec_waste;
            st.ms_setup = std::max(st.ms_setup, x.ms_setup); st.ms_d2h += x.ms_d2h;
        }
        for (uint64_t j = 0; j < std::min<uint64_t>(x.nw_launches, IMSAME_LAUNCH_STATS); ++j) {
            if (st.nw_launches + j >= IMSAME_LAUNCH_STATS) break;
            st.launch_cand[st.nw_launches + j] = x.launch_cand[j]; st.launch_ms[st.nw_launches + j] = x.launch_ms[j];
            if ((x.launch_pk >> j) & 1) st.launch_pk |= 1ull << (st.nw_launches + j);
            if ((x.launch_k5 >> j) & 1) st.launch_k5 |= 1ull << (st.nw_launches + j);
            if ((x.launch_np >> j) & 1) st.launch_np |= 1ull << (st.nw_launches + j);
            if ((x.launch_k19 >> j) & 1) st.launch_k19 |= 1ull << (st.nw_launches + j);
            if ((x.launch_nwp >> j) & 1) st.launch_nwp |= 1ull << (st.nw_launches + j);
            if ((x.launch_k3 >> j) & 1) st.launch_k3 |= 1ull << (st.nw_launches + j);
        }
        st.nw_launches += x.nw_launches;
    }
    st.nw_launch_ms = st.nw_launches ? st.ms_nw / st.nw_launches : 0;
    st.ms_nw_busy = union_ms(iv);
    span_ms(iv, &st.ms_nw_first, &st.ms_nw_last);
    st.lanes = (uint64_t)nl;
    c->paths_split = true; c->paths_n = used[0]; c->paths_on_host = false;
    c->lane_paths.assign(used.begin() + 1, used.end());
    if (np != nl) {                    // pieces: the lanes' buffers hold only their last piece's paths
        c->paths_split = false; c->paths_n = 0; c->lane_paths.clear();
    }
    if (paths_used) *paths_used = base;
    if (p->want_paths && base && !fn) {
        if (base > paths_cap || !paths) { if (ret == IMSAME_OK) ret = IMSAME_E_PATHS; }
        else {
            uint64_t got = 0;
            int rc = imsame_dev_fetch_paths(c, paths, paths_cap, &got);
            if (rc) return rc;
        }
    }
    st.ms_total = now_ms() - t_start;
    if (stats) *stats = st;
    return ret;
}

extern "C" int imsame_dev_fetch_paths(imsame_ctx *c, uint32_t *paths, uint64_t paths_cap, uint64_t *paths_used) {
    if (!c) return IMSAME_E_ARG;
    uint64_t total = c->paths_n;
    if (c->paths_split)
        for (uint64_t u : c->lane_paths) total += u;
    if (paths_used) *paths_used = total;
    if (total > paths_cap) return IMSAME_E_PATHS;
    if (!total) return IMSAME_OK;
    if (!paths) return IMSAME_E_ARG;
    if (c->paths_on_host) {
        memcpy(paths, c->paths_host.data(), c->paths_n * 4);
        return IMSAME_OK;
    }
    HIPCHK(hipSetDevice(c->device));
    if (c->paths_n) HIPCHK(hipMemcpyAsync(paths, c->paths.p, c->paths_n * 4, hipMemcpyDeviceToHost, c->stream));
    uint64_t off = c->paths_n;
    if (c->paths_split)
        for (size_t k = 0; k < c->lane_paths.size(); ++k) {
            const uint64_t u = c->lane_paths[k];
            if (u) HIPCHK(hipMemcpyAsync(paths + off, c->subs[k]->paths.p, u * 4, hipMemcpyDeviceToHost, c->stream));
            off += u;
        }
    HIPCHK(hipStreamSynchronize(c->stream));
    return IMSAME_OK;
}

// Unit-level entry: NW + backtrack + acceptance for explicit (X_k, Y_k) pairs
// (build_alignment, alignmentFunctions.c:210-274), default-or-given params.
// ---------------------------------------------------------------------------
// Database slices (memory-capped multi-pass index).
// A bucket lists its hits in descending position, so cutting the database
// into record ranges from the TOP down splits every bucket into consecutive
// runs: slice 0 (highest records) first.  The reference's visiting order is
// then (window, slice, rank in slice), and the first accepted pair of the
// whole database is the minimum over slices of each slice's first accepted
// pair under that key.  Passes run slice 0, 1, ...; after a read accepts at
// window w, later slices (whose hits in window w come after) scan windows
// < w only.  Results equal one pass over the whole database; each pass holds
// only its slice's index in HBM.
// ---------------------------------------------------------------------------
// imsame_dev_align on the loaded index with the e-value's L_DB set to the
// whole database (the index holds one slice of it), per-read window caps and
// the window of each accepted hit: the building block of database slices
// (below) and of database shards across GPUs (min of (window, shard) keys).
extern "C" int imsame_dev_align_windows(imsame_ctx *c, uint64_t read_from, uint64_t read_to,
                                        uint64_t n_threads_semantic, const imsame_params *p, uint64_t ev_db_len,
                                        const uint64_t *win_start, const uint64_t *win_cap,
                                        imsame_read_result *res, uint64_t *win,
                                        uint32_t *paths, uint64_t paths_cap, uint64_t *paths_used,
                                        imsame_stats *stats) {
    if (!c || !p || (read_to > read_from && (!res || !win))) return IMSAME_E_ARG;
    if (!c->have_index || !c->have_query) return IMSAME_E_STATE;
    if (read_from < c->q_lo || read_to > c->q_hi || read_from > read_to) return IMSAME_E_ARG;
    HIPCHK(hipSetDevice(c->device));
    const uint32_t n = (uint32_t)(read_to - read_from);
    if (c->wcap.ensure((uint64_t)n * 8 + 8) || c->wout.ensure((uint64_t)n * 8 + 8) ||
        (win_start && c->wstart.ensure((uint64_t)n * 8 + 8)))
        return IMSAME_E_OOM;
    if (win_start) HIPCHK(hipMemcpyAsync(c->wstart.p, win_start, (uint64_t)n * 8, hipMemcpyHostToDevice, c->stream));
    if (win_cap) HIPCHK(hipMemcpyAsync(c->wcap.p, win_cap, (uint64_t)n * 8, hipMemcpyHostToDevice, c->stream));
    else         HIPCHK(hipMemsetAsync(c->wcap.p, 0xFF, (uint64_t)n * 8, c->stream));
    HIPCHK(hipMemsetAsync(c->wout.p, 0xFF, (uint64_t)n * 8, c->stream));
    const uint64_t ymax = range_ymax(c, read_from, read_to);
    c->ev_db_len = ev_db_len;
    c->use_wcap = true;
    c->use_wstart = win_start != nullptr;
    int rc = imsame_dev_align(c, read_from, read_to, n_threads_semantic, p, res, paths, paths_cap, paths_used, stats);
    c->ev_db_len = 0;
    c->use_wcap = c->use_wstart = false;
    if (n && (rc == IMSAME_OK || rc == IMSAME_E_READ_TOO_LONG || rc == IMSAME_E_PATHS)) {
        // window of each accepted hit (same read-start logic and cap as the pass)
        SeedLaunch S;
        memset(&S, 0, sizeof S);
        S.db = c->db.as<uint8_t>(); S.db_start = c->db_start.as<uint64_t>(); S.n_db = c->n_db; S.db_len = c->db_len;
        S.dbw = c->dbw.as<uint32_t>(); S.qw = dev_qw(c);
        S.q = dev_q(c); S.q_start = dev_qs(c); S.n_q = c->n_q; S.q_len = c->q_len;
        S.qs_lo = c->q_lo; S.qs_lo_first = c->q_lo_first;
        S.off = c->off.as<uint64_t>(); S.ent = c->ent.as<uint2>(); S.ent_abs = c->ent_abs;
        S.read_from = read_from;
        S.T = n_threads_semantic ? n_threads_semantic : 1;
        S.rpt = (uint64_t)floorl((long double)c->n_q / (long double)S.T);     // IMSAME.c:414
        S.minraw = c->minraw.as<uint64_t>(); S.n_minraw = (uint32_t)ymax + 1;
        S.wcap = c->wcap.as<uint64_t>();
        accept_window_kernel<<<nblk(n, 256), 256, 0, c->stream>>>(S, c->res.as<imsame_read_result>(), n,
                                                                 c->wout.as<uint64_t>());
        HIPCHK(hipGetLastError());
    }
    if (n) HIPCHK(hipMemcpyAsync(win, c->wout.p, (uint64_t)n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return rc;
}

extern "C" int imsame_dev_align_sliced(imsame_ctx *c, const uint8_t *db_seq, uint64_t db_len,
                                       const uint64_t *db_start, uint64_t n_db, const uint8_t *db_brk,
                                       uint64_t slice_bases, uint64_t read_from, uint64_t read_to,
                                       uint64_t n_threads_semantic, const imsame_params *p, imsame_read_result *res,
                                       uint32_t *paths, uint64_t paths_cap, uint64_t *paths_used,
                                       uint64_t *n_slices, imsame_stats *stats) {
    const double t_start = now_ms();
    if (!c || !p || (!res && read_to > read_from) || (n_db && !db_start) || (db_len && !db_seq)) return IMSAME_E_ARG;
    if (!c->have_query) return IMSAME_E_STATE;
    if (read_from < c->q_lo || read_to > c->q_hi || read_from > read_to || n_db == 0 || slice_bases == 0)
        return IMSAME_E_ARG;
    if (p->want_paths && !paths) return IMSAME_E_ARG;
    // the size error aborts the reference at its first e-value pass in visiting
    // order; slices would see such hits out of order, so the sliced path takes
    // only inputs where it cannot fire
    auto rec_end = [&](uint64_t k) { return k + 1 < n_db ? db_start[k + 1] : db_len; };
    uint64_t max_rec = 0, ymax = 0;
    for (uint64_t k = 0; k < n_db; ++k) max_rec = std::max<uint64_t>(max_rec, rec_end(k) - db_start[k]);
    ymax = range_ymax(c, read_from, read_to);
    if (max_rec > p->max_read_size || ymax > p->max_read_size) return IMSAME_E_ARG;
    // slices: record ranges [lo, hi), top down, each <= slice_bases (>= 1 record)
    std::vector<std::pair<uint64_t, uint64_t>> sl;
    for (uint64_t hi = n_db; hi > 0;) {
        uint64_t lo = hi - 1;
        while (lo > 0 && rec_end(hi - 1) - db_start[lo - 1] <= slice_bases) --lo;
        sl.push_back({lo, hi});
        hi = lo;
    }
    if (n_slices) *n_slices = sl.size();
    const uint32_t n = (uint32_t)(read_to - read_from);
    imsame_stats tot;
    memset(&tot, 0, sizeof tot);
    tot.n_reads = n;
    tot.err_read = ~0ull;
    if (paths_used) *paths_used = 0;
    HIPCHK(hipSetDevice(c->device));
    // Two phases.  A: every slice, windows below a band of BAND windows per
    // read -- most reads accept at their first windows, and the smallest
    // (window, slice) key found there is final since every key below the band
    // was examined.  B: the reads A left, from the band on, slice by slice
    // under the caps.  (Without A, slices not holding a read's record would
    // be scanned over all windows before a cap exists.)
    const uint64_t BAND = 8;
    std::vector<uint64_t> cap(n), wstart(n), wout(n);
    for (uint32_t r = 0; r < n; ++r) cap[r] = hqs(c, read_from + r) + IMSAME_FIXED_K - 1 + BAND;
    std::vector<imsame_read_result> tmp(n);
    std::vector<uint64_t> st_rebased;
    std::vector<uint8_t> brk;
    std::vector<uint32_t> acc;
    uint64_t used = 0;
    int ret = IMSAME_OK;
    for (int phase = 0; phase < 2 && ret == IMSAME_OK; ++phase) {
        if (phase == 1) {
            uint64_t left = 0;
            for (uint32_t r = 0; r < n; ++r) {
                const bool done = res[r].status == 1;
                wstart[r] = cap[r];
                cap[r] = done ? 0 : ~0ull;                // accepted in A: final, not scanned again
                left += !done;
            }
            if (!left) break;
        }
        for (size_t k = 0; k < sl.size() && ret == IMSAME_OK; ++k) {
            const uint64_t lo = sl[k].first, hi = sl[k].second;
            const uint64_t base = lo ? db_start[lo] : 0, len = rec_end(hi - 1) - base;
            st_rebased.resize(hi - lo);
            for (uint64_t r = lo; r < hi; ++r) st_rebased[r - lo] = db_start[r] - base;
            const uint8_t *bk = nullptr;
            if (db_brk && len) {                          // bits [base, base + len) of the bitmap
                brk.assign((len + 7) / 8, 0);
                const uint64_t b0 = base >> 3, sh = base & 7, nsrc = (db_len + 7) / 8;
                for (uint64_t i = 0; i < brk.size(); ++i) {
                    const uint32_t a = b0 + i < nsrc ? db_brk[b0 + i] : 0, b = b0 + i + 1 < nsrc ? db_brk[b0 + i + 1] : 0;
                    brk[i] = (uint8_t)(sh ? ((a >> sh) | (b << (8 - sh))) : a);
                }
                bk = brk.data();
            }
            int rc = imsame_dev_index(c, db_seq + base, len, st_rebased.data(), hi - lo, bk);
            if (rc) return rc;
            imsame_stats st;
            uint64_t pu = 0;
            // this slice's paths are appended to the host-side arena acc
            rc = imsame_dev_align_windows(c, read_from, read_to, n_threads_semantic, p, db_len,
                                          phase ? wstart.data() : nullptr, cap.data(), tmp.data(), wout.data(),
                                          nullptr, 0, &pu, &st);
            if (rc == IMSAME_E_PATHS) {
                acc.resize(used + pu);
                rc = imsame_dev_fetch_paths(c, acc.data() + used, pu, &pu);
            }
            if (rc) { ret = rc; break; }
            tot.n_rewalk += st.n_rewalk; tot.nw_redo += st.nw_redo;
            tot.n_nw += st.n_nw; tot.nw_cells += st.nw_cells; tot.n_hits += st.n_hits; tot.rounds += st.rounds;
            tot.ms_seed += st.ms_seed; tot.ms_nw += st.ms_nw; tot.nw_launches += st.nw_launches;
            tot.nw_bytes += st.nw_bytes;
            for (uint32_t r = 0; r < n; ++r) {
                if (phase == 0 && k == 0) res[r] = tmp[r];  // not found (ylen) unless a slice accepts
                if (tmp[r].status != 1) continue;
                if (wout[r] >= cap[r]) return IMSAME_E_STATE;   // cannot happen: the pass scanned below the cap
                res[r] = tmp[r];
                res[r].db_seq += lo;
                res[r].path_off += (uint32_t)used;
                cap[r] = wout[r];
            }
            used += pu;
        }
    }
    c->paths_host.swap(acc);
    c->paths_n = used; c->paths_on_host = true;
    if (paths_used) *paths_used = used;
    if (p->want_paths && ret == IMSAME_OK) {
        if (used > paths_cap) ret = IMSAME_E_PATHS;                  // imsame_dev_fetch_paths
        else if (used) memcpy(paths, c->paths_host.data(), used * 4);
    }
    for (uint32_t r = 0; r < n; ++r) tot.n_accepted += res[r].status == 1;
    tot.nw_launch_ms = tot.nw_launches ? tot.ms_nw / tot.nw_launches : 0;
    tot.ms_total = now_ms() - t_start;
    if (stats) *stats = tot;
    return ret;
}

extern "C" int imsame_dev_nw_pairs(imsame_ctx *c, const uint8_t *xs, const uint64_t *x_start, const uint8_t *ys,
                                   const uint64_t *y_start, uint64_t npairs, const imsame_params *p,
                                   imsame_read_result *res, uint32_t *paths, uint64_t paths_cap, uint64_t *paths_used,
                                   double *kernel_ms) {
    if (!c || !p || !res || npairs == 0) return IMSAME_E_ARG;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const uint64_t xl = x_start[npairs], yl = y_start[npairs];
    uint32_t xmax = 0, ymax = 0;
    for (uint64_t k = 0; k < npairs; ++k) {
        xmax = (uint32_t)std::max<uint64_t>(xmax, x_start[k + 1] - x_start[k]);
        ymax = (uint32_t)std::max<uint64_t>(ymax, y_start[k + 1] - y_start[k]);
        if (x_start[k + 1] - x_start[k] < 2 || y_start[k + 1] - y_start[k] < 2) return IMSAME_E_ARG;
    }
    if (!imsame_gaps_in_range(p->igap, p->egap, xmax, ymax)) return IMSAME_E_RANGE;
    if (std::max(xmax, ymax) > 0x3FFF) return IMSAME_E_ARG;
    DBuf dx, dxs, dy, dys, dc, dout;
    if (dx.ensure(xl + 64) || dxs.ensure((npairs + 1) * 8) || dy.ensure(yl + 64) || dys.ensure((npairs + 1) * 8) ||
        dc.ensure(npairs * 8) || dout.ensure(npairs * 64))
        return IMSAME_E_OOM;
    std::vector<uint32_t> idx(npairs);
    for (uint64_t k = 0; k < npairs; ++k) idx[k] = (uint32_t)k;
    HIPCHK(hipMemcpyAsync(dx.p, xs, xl, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(dxs.p, x_start, (npairs + 1) * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(dy.p, ys, yl, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(dys.p, y_start, (npairs + 1) * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(dc.p, idx.data(), npairs * 4, hipMemcpyHostToDevice, s));
    uint64_t saved = c->db_len;
    c->db_len = 1;     // e-value table unused here
    int rc = build_tables(c, p, ymax, xmax);
    c->db_len = saved;
    if (rc) return rc;
    uint32_t pcap = 0;
    if ((rc = paths_setup(c, p, paths_cap, &pcap))) return rc;
    uint64_t *ctr = c->ctr.as<uint64_t>();
    HIPCHK(hipMemsetAsync(ctr, 0, C_NSLOTS * 8, s));
    NwPlan pl;
    bool ymult = true, yuni = true;
    for (uint64_t k = 0; k < npairs; ++k) {
        ymult = ymult && (y_start[k + 1] - y_start[k]) % NW16_K == 0;
        yuni = yuni && y_start[k + 1] - y_start[k] == ymax;
    }
    if ((rc = plan_nw(c, ymax, xmax, (uint32_t)npairs, p, ymult, &pl, false, yuni ? ymax : 0))) return rc;
    double ms = 0;
    rc = launch_nw(c, pl, dc.as<uint32_t>(), dc.as<uint32_t>(), (uint32_t)npairs, dout.as<imsame_read_result>(),
                   p->igap, p->egap, p, ymax, xmax, (uint32_t *)(ctr + C_WORK), dx.as<uint8_t>(), dxs.as<uint64_t>(),
                   dy.as<uint8_t>(), dys.as<uint64_t>(), pcap, &ms);
    if (rc) return rc;
    if (kernel_ms) *kernel_ms = ms;
    HIPCHK(hipMemcpyAsync(res, dout.p, npairs * 64, hipMemcpyDeviceToHost, s));
    uint64_t hc[C_NSLOTS];
    HIPCHK(hipMemcpyAsync(hc, ctr, C_NSLOTS * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (getenv("IMSAME_NW_PROF") && pl.pk) {  // diagnostics (scripts/micro/nw16_loop.py): raw phase wave-cycles
        fprintf(stderr, "[nwprof-raw] blocks %u G %d GPW %d k %d steps %d cand %llu setup %llu sweep1 %llu reduce %llu "
                "sweep2 %llu walk %llu rt %llu ms %.4f\n", pl.blocks, pl.G, pl.GPW, pl.k, pl.steps,
                (unsigned long long)npairs, (unsigned long long)hc[C_PROF], (unsigned long long)hc[C_PROF + 1],
                (unsigned long long)hc[C_PROF + 2], (unsigned long long)hc[C_PROF + 3], (unsigned long long)hc[C_PROF + 4],
                (unsigned long long)hc[C_PROF + 5], ms);
    }
    if (getenv("IMSAME_NW_PROF") && pl.lng)   // diagnostics: which long-read kernel, waves that fell back
        fprintf(stderr, "[nwprof-long] kernel %s blocks %u cand %llu fallback %llu ms %.4f\n",
                pl.lp ? "nwp" : "nwl", pl.blocks, (unsigned long long)npairs, (unsigned long long)hc[C_FBK], ms);
    int ret = IMSAME_OK;
    if (p->want_paths) {
        if (paths_used) *paths_used = (uint32_t)hc[C_PATHS];
        if (hc[C_FLAGS] & 1) ret = IMSAME_E_PATHS;
        else if (hc[C_PATHS]) {
            HIPCHK(hipMemcpyAsync(paths, c->paths.p, (uint32_t)hc[C_PATHS] * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        }
    }
    dx.release(); dxs.release(); dy.release(); dys.release(); dc.release(); dout.release();
    return ret;
}

// reverseComplement.c:21-118 on the device (see revcomp_kernel.hip)
extern "C" int imsame_dev_revcomp(imsame_ctx *c, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap,
                                  uint64_t *out_len) {
    if (!c || !out_len || (n && !in)) return IMSAME_E_ARG;
    if (n >= 0xFFFFFFF0ull) return IMSAME_E_ARG;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    *out_len = 0;
    if (n == 0) return IMSAME_OK;
    if (c->rc_in.ensure(n + 16) || c->rc_a.ensure((n + 1) * 4 * 2 + 64) || c->rc_b.ensure((n + 1) * 4 * 2 + 64))
        return IMSAME_E_OOM;
    uint32_t *fgt = c->rc_a.as<uint32_t>(), *flet = fgt + (n + 1);
    uint32_t *gpos = c->rc_b.as<uint32_t>(), *let = gpos + (n + 1);
    HIPCHK(hipMemcpyAsync(c->rc_in.p, in, n, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(fgt, 0, (n + 1) * 4 * 2, s));
    rc_flags<<<nblk(n, 256), 256, 0, s>>>(c->rc_in.as<uint8_t>(), n, fgt, flet);
    int rc = dev_scan(s, fgt, gpos, n + 1);
    if (!rc) rc = dev_scan(s, flet, let, n + 1);
    if (rc) return rc;
    uint32_t nr = 0;
    HIPCHK(hipMemcpyAsync(&nr, gpos + n, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (nr == 0) return IMSAME_OK;
    // output offsets and sizes are u32: a record's output is at most its input
    // bytes + one '\n' (headers copied, bodies lose their newlines), so the
    // whole output is < n + nr; refuse what could wrap instead of wrapping
    if ((uint64_t)n + nr >= 0xFFFFFFF0ull) return IMSAME_E_ARG;
    if (c->rc_c.ensure((uint64_t)nr * 4 * 5 + 64)) return IMSAME_E_OOM;
    if ((rc = c->rc_c.poison(s)) || (rc = c->rc_out.poison(s))) return rc;
    uint32_t *off = c->rc_c.as<uint32_t>(), *hend = off + nr, *bend = hend + nr, *szr = bend + nr, *oo = szr + nr;
    rc_offsets<<<nblk(n, 256), 256, 0, s>>>(c->rc_in.as<uint8_t>(), n, gpos, off);
    rc_records<<<nblk(nr, 256), 256, 0, s>>>(c->rc_in.as<uint8_t>(), n, off, nr, let, hend, bend, szr);
    // sizes can exceed 2^32 only for > 4 GB outputs (rejected above for inputs)
    DBuf oo1;
    if (oo1.ensure(((uint64_t)nr + 1) * 4)) return IMSAME_E_OOM;
    HIPCHK(hipMemsetAsync(oo1.p, 0, ((uint64_t)nr + 1) * 4, s));
    HIPCHK(hipMemcpyAsync(oo1.p, szr, (uint64_t)nr * 4, hipMemcpyDeviceToDevice, s));
    if ((rc = dev_scan(s, oo1.as<uint32_t>(), oo, nr))) return rc;
    uint32_t last_o = 0, last_sz = 0;
    HIPCHK(hipMemcpyAsync(&last_o, oo + nr - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&last_sz, szr + nr - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const uint64_t total = (uint64_t)last_o + last_sz;
    *out_len = total;
    if (total > out_cap || !out) return IMSAME_E_ARG;
    if (c->rc_out.ensure(total + 16)) return IMSAME_E_OOM;
    rc_headers<<<nblk(nr, 256), 256, 0, s>>>(c->rc_in.as<uint8_t>(), off, nr, hend, bend, let, oo, c->rc_out.as<uint8_t>());
    rc_bodies<<<nblk(n, 256), 256, 0, s>>>(c->rc_in.as<uint8_t>(), n, off, nr, hend, bend, let, oo, c->rc_out.as<uint8_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, c->rc_out.p, total, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    oo1.release();
    return IMSAME_OK;
}
