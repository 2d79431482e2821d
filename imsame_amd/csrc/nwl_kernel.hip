// nwl_kernel.hip -- IMSAME's NW + backtracking for LONG reads (longer than the
// packed kernel's 160 columns): one candidate per wave, two passes.  Included
// by imsame_dev.hip (and by tests/emu/wave_emu.cpp under IMSAME_WAVE_EMU) after
// nw_kernel.hip and nw16_kernel.hip.
//
// Reference: NW              alignmentFunctions.c:389-489
//            backtrackingNW  alignmentFunctions.c:493-560
//
// Mapping.  The read's columns are cut into strips of NWL_W = 640; lane l owns
// NWL_K = 10 consecutive columns of a strip and walks the rows with a
// one-lane skew (step t: row i = t - l).  The row state (T, mf score, left
// term) crosses lanes by DPP wave_shr:1 and strips through a seam: the
// strip's last lane writes its right edge per row, the next strip's lead lane
// reads it.  Int32 values with nw16_kernel.hip's recurrence: the gap terms are
// DRIFTING state (l0 += eg per column, u0 += eg per row, re-based on a take)
// and the column maximum lives in the +ig+eg frame, so a cell costs no
// per-column or per-row constant.
//
// Pass 1, score only, strip after strip: each strip's seam is kept (3 ints per
// row), and every NWL_CK steps the wave's registers (NWL_NST dwords per lane)
// are saved; the best cell (last row / last column, ">=": the last visited
// wins) comes out of it.  No traceback is written: the int32 kernel
// (nw_kernel.hip) stores 4 bits for every one of a 10 kbp x 12 kbp matrix's
// 120M cells (99 MB per wave slot, the HBM arena capping residency).
// Pass 2 is backtrackingNW's walk from the best cell.  Every cell it reads
// lies in a (strip, step) BAND that is recomputed from the checkpoint below it
// -- the very state pass 1 had, so the very values -- this time with
// nw_kernel.hip's traceback nibble per cell (move, U, L).  A band holds up to
// NWL_BAND steps ending at the cell asked for; the walk moves up and left only,
// so it asks for the next band when it leaves the strip or the band's top (a
// diagonal path: about one band per strip).  Jump sources are searched as in
// nw_walk (the last U above in the column, the last L to the left in the
// row), a search that leaves the band resuming where it stopped.
#include "wave_ops.h"

#define NWL_K    10                       // columns per lane (<= 16: two traceback words)
#define NWL_W    (64 * NWL_K)             // columns per strip
#define NWL_BIG  (1 << 28)                // stands for INT64_MIN / "never"
#define NWL_CK   128                      // checkpoint interval (steps; even: the rotation period)
#define NWL_NST  (4 * NWL_K + 5)          // dwords of wave state per lane in a checkpoint
#define NWL_BAND 1024                     // most steps a pass-2 band ends with (plus up to NWL_CK below)
#define NWL_BAND_DEF 768                  // the default: a diagonal path crosses a strip in ~W + 64 steps

// the long kernel takes launches of reads longer than the packed kernel's
// columns with non-positive gap parameters (the drifting terms only fall)
__host__ static inline bool nwl_fits(int64_t ig, int64_t eg, uint64_t ymax) {
    return ig <= 0 && eg <= 0 && ymax > (uint64_t)NW_W / 2;
}

// Launch shape: one candidate per wave; xstride = LDS bytes of the record
// packed four 2-bit codes per byte.
__host__ static inline NwShape nwl_shape(uint32_t ymax, uint32_t xcap) {
    NwShape s;
    s.G = 64; s.GPW = 1;
    s.nstr = (int)((ymax + NWL_W - 1) / NWL_W);
    if (s.nstr < 1) s.nstr = 1;
    s.xcap = xcap < 2 ? 2 : (int)xcap;
    s.xstride = ((s.xcap + 3) / 4 + 16 + 15) & ~15;
    s.steps = s.xcap + 64;
    return s;
}
__host__ __device__ static inline int nwl_ncks(int steps) { return (steps + NWL_CK - 1) / NWL_CK + 1; }
// per wave slot: checkpoints (ck arena), seams (bnd arena), band traceback +
// path scratch (tb arena)
__host__ static inline uint64_t nwl_ck_words(const NwShape &s) {
    return (uint64_t)s.nstr * nwl_ncks(s.steps) * NWL_NST * 64;
}
__host__ static inline uint64_t nwl_seam_words(const NwShape &s) { return (uint64_t)s.nstr * (s.xcap + 1) * 3; }
__host__ __device__ static inline uint64_t nwl_band_words() { return (uint64_t)(NWL_BAND + NWL_CK + 64) * 64 * 2; }
// pass 2: band + path scratch; pass 1: the last column's strip cells (K per row)
__host__ static inline uint64_t nwl_tb_words(const NwShape &s, uint32_t ymax) {
    return std::max<uint64_t>(nwl_band_words() + (uint64_t)s.xcap + ymax + 64, (uint64_t)s.xcap * NWL_K + 64);
}
// LDS per wave: the packed record, the last row of a strip (K ints per lane;
// later the best-cell reduction)
__host__ __device__ static inline size_t nwl_wave_lds(int xstride) { return (size_t)xstride + 64 * NWL_K * 4; }

WV_DEVICE uint32_t nwl_code(const uint8_t *X4, int i) { return (X4[i >> 2] >> (2 * (i & 3))) & 3u; }

// one lane's view of the walk's band: strip bst, steps [bt0, bt1)
struct NwlBand {
    const uint32_t *tb; const uint8_t *X4; const uint8_t *Y;
    int bst, bt0, bt1;
    __device__ bool has(int i, int j) const {
        const int st = j / NWL_W, l = (j - st * NWL_W) / NWL_K, t = i + l;
        return st == bst && t >= bt0 && t < bt1;
    }
    __device__ uint32_t nib(int i, int j) const {
        const int jj = j - bst * NWL_W, l = jj / NWL_K, s = jj - l * NWL_K, t = i + l;
        const uint32_t w = tb[((uint32_t)(t - bt0) * 64u + (uint32_t)l) * 2u + (uint32_t)(s >> 3)];
        // cells shift in from the bottom, 4 bits each (not-diag, up > left, U,
        // L): word 0 holds cells 0-7, word 1 cells 8..K-1, the first cell on top
        const int top = (s < 8) ? 4 * min(NWL_K, 8) - 1 - 4 * s : 4 * (NWL_K - 8) - 1 - 4 * (s - 8);
        const uint32_t v = (w >> (top - 3)) & 0xFu;     // bit 3 = not-diag ... bit 0 = L
        // -> nw_kernel.hip's nibble: move (0 diag, 1 up, 2 left) | U << 2 | L << 3
        return ((v & 8u) ? ((v & 4u) ? 1u : 2u) : 0u) | ((v & 2u) << 1) | ((v & 1u) << 3);
    }
    __device__ bool match(int i, int j) const { return nwl_code(X4, i) == base_code(Y[j]); }
};

// The walk (backtrackingNW, :493-560) as a resumable state: walk_band runs it
// on the band it is given until the path ends, goes bad, or needs a cell the
// band does not hold (need_i, need_j) -- a diagonal run, an up-search of
// column py (rows sb, sb-1, ...) or a left-search of row px (columns sb, ...)
// stops exactly there and resumes after the next band.  Path entries go to
// `path` (lane 0) as nw_walk emits them.
struct NwlWalk {
    int px, py, len, idn, ig, eg, nent, run, mode, sb, need_i, need_j;
    bool bad, done, need;
};

// (Band: NwlBand here, NwpBand for the packed long kernel -- has / nib / match)
template <class Band>
__device__ void nwl_walk_band(const Band &bd, NwlWalk &w, const int lane, uint32_t *path, int &guard) {
    w.need = false;
    while (!w.done && !w.bad && !w.need) {
        if (w.px <= 0 || w.py <= 0) { w.done = true; break; }
        if (--guard < 0) { w.bad = true; break; }
        int src = -1;
        bool is_up = false;
        if (w.mode == 0) {                       // diagonal run: 64 cells at once
            const int cx = w.px - lane, cy = w.py - lane;
            const bool valid = cx >= 1 && cy >= 1;
            const bool av = valid && bd.has(cx, cy);
            uint32_t nib = 0xFu;
            bool m = false;
            if (av) { nib = bd.nib(cx, cy); m = bd.match(cx, cy); }
            const unsigned long long bs = wv_ballot(!av || (nib & 3u) != 0), bm = wv_ballot(av && m),
                                     bl = wv_ballot(valid && !av);
            const int first = bs ? __builtin_ctzll(bs) : 64;
            const unsigned long long below = first >= 64 ? ~0ull : ((1ull << first) - 1);
            const uint32_t mvj = (uint32_t)wv_shfl((int)(nib & 3u), first < 64 ? first : 0);
            if (first > 0) {
                if (!w.run) w.nent++;
                w.run += first;
                w.len += first; w.idn += __builtin_popcountll(bm & below);
                w.px -= first; w.py -= first;
            }
            if (first >= 64 || w.px <= 0 || w.py <= 0) continue;
            if ((bl >> first) & 1ull) { w.need = true; w.need_i = w.px; w.need_j = w.py; break; }
            if (mvj == 1u) { w.mode = 1; w.sb = w.px - 1; }
            else if (mvj == 2u) { w.mode = 2; w.sb = w.py - 1; }
            else { w.bad = true; break; }
            continue;
        }
        if (w.mode == 1) {                       // up: last row r < px of column py with U -> source r - 2
            const int r = w.sb - lane;
            const bool ok = r >= 1, av = ok && bd.has(r, w.py);
            const bool u = av && ((bd.nib(r, w.py) >> 2) & 1u);
            const unsigned long long gb = wv_ballot(u), gm = wv_ballot(ok && !av);
            if (gm && (!gb || __builtin_ctzll(gm) < __builtin_ctzll(gb))) {
                w.sb -= __builtin_ctzll(gm);                      // rows above sb held no U
                w.need = true; w.need_i = w.sb; w.need_j = w.py;
                break;
            }
            if (gb) src = w.sb - __builtin_ctzll(gb) - 2;
            else if (w.sb - 64 < 1) src = 0;
            else { w.sb -= 64; continue; }
            is_up = true;
        } else {                                 // left: last column c < py of row px with L -> source c - 1
            const int c = w.sb - lane;
            const bool ok = c >= 1, av = ok && bd.has(w.px, c);
            const bool lb = av && ((bd.nib(w.px, c) >> 3) & 1u);
            const unsigned long long gb = wv_ballot(lb), gm = wv_ballot(ok && !av);
            if (gm && (!gb || __builtin_ctzll(gm) < __builtin_ctzll(gb))) {
                w.sb -= __builtin_ctzll(gm);
                w.need = true; w.need_i = w.px; w.need_j = w.sb;
                break;
            }
            if (gb) src = w.sb - __builtin_ctzll(gb) - 1;
            else if (w.sb - 64 < 1) { w.bad = true; break; }     // L(i, 1) is always set
            else { w.sb -= 64; continue; }
        }
        int n;
        if (is_up) { n = w.px - src; w.px = src; w.py -= 1; }   // X run vs '-'  (:520-530)
        else       { n = w.py - src; w.py = src; w.px -= 1; }   // '-' vs Y run  (:531-543)
        if (n < 1) { w.bad = true; break; }
        if (lane == 0 && path) {
            if (w.run) path[w.nent - 1] = (IMSAME_MOVE_DIAG << 30) | (uint32_t)w.run;
            path[w.nent] = ((is_up ? IMSAME_MOVE_UP : IMSAME_MOVE_LEFT) << 30) | (uint32_t)n;
        }
        w.nent++;
        w.run = 0;
        w.len += n; w.eg += n - 1; w.ig += 1;
        w.mode = 0;
    }
}

// candidate c, start to finish (its own LDS record, seams, checkpoints, band)
__device__ void nwl_cand(const NwLaunch &P, uint8_t *wsm, const int lane, const uint32_t slot, const uint32_t c) {
    constexpr int K = NWL_K;
    const int ig = P.igap, eg = P.egap, IGE = ig + eg;
    uint8_t *X4 = wsm;
    int *lrow = (int *)(wsm + P.xstride);                              // 64 lanes x K ints
    int *red = lrow;                                                   // 64 lanes x 4 ints, after pass 1
    uint32_t *tbw = P.tb + (uint64_t)slot * P.tb_wave_dw;              // band traceback, then path scratch
    uint32_t *pscr = tbw + nwl_band_words();
    int *colbuf = (int *)tbw;                                          // pass 1: row i's last-lane cells at i * K
    int *seam = P.bnd + (uint64_t)slot * P.bnd_wave;
    uint32_t *ckw = P.ck + (uint64_t)slot * P.ck_wave_dw + lane;
    const int ncks = nwl_ncks(P.steps);
    const int band = (P.band_w > 0 && P.band_w < NWL_BAND) ? P.band_w : NWL_BAND;   // tests: small bands
    {
        const uint32_t rd = P.cand_read[c], sid = P.cand_sid[c];
        const uint64_t xo = P.db_start[sid];
        const int xlen = (int)(P.db_start[sid + 1] - xo);
        const uint64_t yo = P.q_start[rd];
        const int ylen = (int)(P.q_start[rd + 1] - yo);
        const uint8_t *Xg = P.db + xo, *Y = P.q + yo;
        // the record in LDS, four 2-bit codes per byte (base_code: A0 C1 T2 G3)
        for (int b = lane; b < (xlen + 3) / 4; b += 64) {
            uint32_t v = 0;
            for (int k = 0; k < 4; ++k) v |= base_code(Xg[min(4 * b + k, xlen - 1)]) << (2 * k);
            X4[b] = (uint8_t)v;
        }
        wv_lds_sync();
        const int nstr = (ylen + NWL_W - 1) / NWL_W, xl1 = max(xlen - 1, 0);
        const int tend = xlen - 1 + 64;           // the last lane's last row at step tend - 1
        const int lastst = (ylen - 1) / NWL_W, lastl = ((ylen - 1) - lastst * NWL_W) / K,
                  lasts = (ylen - 1) - lastst * NWL_W - lastl * K;
        int bestR = INT_MIN, bestRj = 0, bestC = INT_MIN, bestCi = 0;

        // ---- state of one strip's sweep, shared by both passes
        const int SP = xlen + 1;                  // seam plane stride: rows 0..xlen
        uint32_t yreg[K];
        int A[K], B[K], mcS[K], u0[K];
        int I1 = 0, I2 = 0, outT = 0, outMS = 0, outL = 0;
        // score tables (v_perm sources: byte y = s(x, y), byte 4 + y its sign)
        // of this lane's row (tL, tH) and of the block's rows, lane l = row
        // t_b + l (xL, xH): every step the lead lane pops the next row's table
        // and the other lanes take their left neighbour's
        uint32_t tL = 0, tH = 0, xL = 0, xH = 0;
        // the previous strip's right edge: R = this block's rows (lane l = row
        // t_b + l, popped by the lead lane), N = the next block's (in flight);
        // W collects the last lane's edge, flushed every block
        int R0 = 0, R1 = 0, R2 = 0, N0 = 0, N1 = 0, N2 = 0, W0 = 0, W1 = 0, W2 = 0;
        int st = 0;
        bool leadc0 = false, seam_in = false, seam_out = false;
        const int *seam_rd = seam;
        int *seam_wr = seam;
        uint32_t *tbb = tbw;
        int bt0 = 0;
        auto row_table = [&](const int r, uint32_t &L, uint32_t &H) {
            const uint32_t xs = nwl_code(X4, min(max(r, 0), xl1)) * 0x01010101u;
            L = wv_perm(NW16_TBL_HI, NW16_TBL_LO, xs ^ 0x03020100u);
            H = wv_perm(NW16_TBL_HI, NW16_TBL_LO, xs ^ 0x07060504u);
        };
        auto seam_load = [&](const int r0) {      // edge rows r0 + lane (clamped into [1, xlen))
            const int r = min(max(r0 + lane, 1), xl1);
            N0 = seam_rd[r]; N1 = seam_rd[SP + r]; N2 = seam_rd[2 * SP + r];
        };
        auto seam_flush = [&](const int t, const int ts) {   // W = steps [t - 64, t): lane l row t - 127 + l
            const int r = t - 127 + lane;
            if (r >= 1 && r < xlen && r >= ts - 63) { seam_wr[r] = W0; seam_wr[SP + r] = W1; seam_wr[2 * SP + r] = W2; }
        };
        // strip setup: y codes, row 0 (:404-413), the flags of this strip
        auto strip_init = [&](const int s_) {
            st = s_;
            const int j0 = st * NWL_W + lane * K;
            leadc0 = st == 0 && lane == 0;
            seam_in = st > 0;
            seam_out = st + 1 < nstr;
            seam_rd = seam + (uint64_t)(st > 0 ? st - 1 : 0) * 3 * SP;
            seam_wr = seam + (uint64_t)st * 3 * SP;
            const uint32_t x0 = nwl_code(X4, 0), xs0 = x0 * 0x01010101u;
#pragma unroll
            for (int s = 0; s < K; ++s) {
                const uint32_t y = (j0 + s < ylen) ? base_code(Y[j0 + s]) : 0u;
                yreg[s] = y | ((y | 4u) << 8) | ((y | 4u) << 16) | ((y | 4u) << 24);
                A[s] = (int)wv_perm(NW16_TBL_HI, NW16_TBL_LO, xs0 ^ yreg[s]);
                B[s] = A[s];
            }
            const uint32_t yp = j0 > 0 ? base_code(Y[min(j0 - 1, ylen - 1)]) : 0u;
            const int t0prev = (int)wv_perm(NW16_TBL_HI, NW16_TBL_LO,
                                            xs0 ^ (yp | ((yp | 4u) << 8) | ((yp | 4u) << 16) | ((yp | 4u) << 24)));
#pragma unroll
            for (int s = 0; s < K; ++s) {
                // mc[j-1] = (T[0][j-1], row 0); row 0 stands in for rows -1 and -2
                mcS[s] = ((s == 0) ? t0prev : A[s - 1]) + IGE;
                u0[s] = mcS[s];
                if (j0 + s == 1) mcS[s] = NWL_BIG;          // mc[0] is never updated (:476)
            }
            I1 = t0prev; I2 = t0prev;
            outT = A[K - 1]; outMS = 0; outL = 0;
        };
        // one step of the sweep (roles (cur, own) swap every step): HEAD = some
        // lane may be at row <= 1; TAIL = rows may pass the record's end; TB =
        // write the traceback nibbles (pass 2, band step t - bt0); BEST = track
        // the last row / last column (pass 1)
        auto step = [&](const bool HEAD, const bool TAIL, const bool TB, const bool BEST, const int t, int (&cur)[K],
                        const int (&own)[K], int &in0, const int in1) {
            // row state from the left neighbour; the lead lane's from the
            // previous strip's edge (strip 0: unused, column 0 below)
            // (each queue shifts before its head is consumed as the DPP's old
            // value, so the consumer takes over the head's register: no copies)
            const int R0n = wv_shl1(R0), R1n = wv_shl1(R1), R2n = wv_shl1(R2);
            const int sN = wv_shr1_fill(outT, R0), mS = wv_shr1_fill(outMS, R1), mL0 = wv_shr1_fill(outL, R2);
            R0 = R0n; R1 = R1n; R2 = R2n;
            const uint32_t xLn = (uint32_t)wv_shl1((int)xL), xHn = (uint32_t)wv_shl1((int)xH);
            tL = (uint32_t)wv_shr1_fill((int)tL, (int)xL); tH = (uint32_t)wv_shr1_fill((int)tH, (int)xH);
            xL = xLn; xH = xHn;
            const int i = t - lane;
            const bool pre = HEAD && i < 1;
            const bool row1 = HEAD && i <= 1;         // up invalid, mc frozen (:449, :476)
            int mfS = mS, l0 = mL0;
            int dIn = in0 + IGE;                      // T[i-2][j-1] + ig + eg: cur before this step overwrites it
            uint32_t w0 = 0, w1 = 0;
#pragma unroll
            for (int s = 0; s < K; ++s) {
                const int d0 = (s == 0) ? in1 : own[s - 1];      // T[i-1][j-1]
                const int tl = (s == 0) ? sN : cur[s - 1];       // T[i][j-1]
                const int dI = dIn;
                dIn = cur[s] + IGE;
                const int sc = (int)wv_perm(tH, tL, yreg[s]);
                const int up = row1 ? -NWL_BIG : u0[s];
                int v;
                uint32_t &tw = (s < 8) ? w0 : w1;
                if (TB) {
                    // diag if >= both, else up if up > left, else left (:457-472)
                    const int lu = max(l0, up);
                    v = max(d0, lu) + sc;
                    tw = wv_shift_in(tw, d0 < lu);
                    tw = wv_shift_in(tw, up > l0);
                } else {
                    v = wv_max3(d0, l0, up) + sc;
                }
                if (s == 0 && leadc0) v = sc;                    // column 0 (:426)
                cur[s] = pre ? own[s] : v;
                // column max of column j-1 over rows <= i-2, strict > (:476-480), in
                // the +ig+eg frame: dI = T[i-2][j-1] + ig + eg
                const bool mU = mcS[s] < dI;
                const int u0n = (mU ? dI : u0[s]) + eg;
                u0[s] = row1 ? u0[s] : u0n;
                mcS[s] = mU ? dI : mcS[s];
                // row state for column j+1: tested on row i, taken from row i-1 (:434-438)
                const bool kept = tl < mfS;
                l0 = kept ? l0 + eg : d0 + IGE;
                mfS = kept ? mfS : d0;
                if (s == 0 && leadc0) { mfS = -NWL_BIG; l0 = -NWL_BIG; }   // j = 1: no left move
                if (TB) {
                    tw = wv_shift_in(tw, mU);
                    tw = wv_shift_in(tw, !kept);
                }
            }
            if (TB) {                                 // rows outside [1, xlen) are never read
                uint32_t *rec = tbb + ((uint32_t)(t - bt0) * 64u + (uint32_t)lane) * 2u;
                rec[0] = w0; rec[1] = w1;
            }
            if (BEST) {
                if (TAIL && i == xlen - 1) {          // last row: kept for the strip's end (last_row)
#pragma unroll
                    for (int s = 0; s < K; ++s) lrow[lane * K + s] = cur[s];
                }
                if (st == lastst && lane == lastl && i >= 1 && i < xlen - 1) {     // last column: kept (colbuf)
                    int *q = colbuf + (uint32_t)i * K;
#pragma unroll
                    for (int s = 0; s < K; ++s) q[s] = cur[s];
                }
            }
            if (seam_out) {                           // the last lane's edge, row i, into W
                W0 = wv_shl1_fill(W0, cur[K - 1]); W1 = wv_shl1_fill(W1, mfS); W2 = wv_shl1_fill(W2, l0);
            }
            in0 = pre ? in1 : sN;
            outT = cur[K - 1]; outMS = mfS; outL = l0;
        };
        // checkpoint m of strip st: the state before step 1 + m*NWL_CK, roles (A, B), (I2, I1)
        auto save = [&](const int m) {
            uint32_t *p = ckw + (uint32_t)((st * ncks + m) * NWL_NST) * 64u;
#pragma unroll
            for (int s = 0; s < K; ++s) {
                p[s * 64] = (uint32_t)A[s]; p[(K + s) * 64] = (uint32_t)B[s];
                p[(2 * K + s) * 64] = (uint32_t)mcS[s]; p[(3 * K + s) * 64] = (uint32_t)u0[s];
            }
            p[4 * K * 64] = (uint32_t)I1; p[(4 * K + 1) * 64] = (uint32_t)I2;
            p[(4 * K + 2) * 64] = (uint32_t)outT; p[(4 * K + 3) * 64] = (uint32_t)outMS;
            p[(4 * K + 4) * 64] = (uint32_t)outL;
        };
        auto restore = [&](const int m) {
            const uint32_t *p = ckw + (uint32_t)((st * ncks + m) * NWL_NST) * 64u;
#pragma unroll
            for (int s = 0; s < K; ++s) {
                A[s] = (int)p[s * 64]; B[s] = (int)p[(K + s) * 64];
                mcS[s] = (int)p[(2 * K + s) * 64]; u0[s] = (int)p[(3 * K + s) * 64];
            }
            I1 = (int)p[4 * K * 64]; I2 = (int)p[(4 * K + 1) * 64];
            outT = (int)p[(4 * K + 2) * 64]; outMS = (int)p[(4 * K + 3) * 64]; outL = (int)p[(4 * K + 4) * 64];
        };
        // run steps [ts, t1) from the state before step ts (ts = 1 mod NWL_CK)
        // in blocks of 64 steps; within a block the head (rows <= 1
        // somewhere), the middle, the tail (rows past the record)
        auto sweep = [&](const int ts, const int t1, const bool TB, const bool BEST, const bool CKS) {
            row_table(ts - 1 - lane, tL, tH);         // as the left neighbour would hand it over
            if (seam_in) seam_load(ts);
            const int head_end = 66, tail_beg = xlen - 2;          // fast steps: every lane in rows [2, xlen - 1)
            int t = ts;
            while (t < t1) {
                if (CKS && (t - 1) % NWL_CK == 0) save((t - 1) / NWL_CK);
                row_table(t + lane, xL, xH);
                if (seam_in) { R0 = N0; R1 = N1; R2 = N2; seam_load(t + 64); }
                if (seam_out && t > ts) seam_flush(t, ts);
                const int te = min(t + 64, t1);
                for (; t + 1 < te && t + 1 < head_end; t += 2) {
                    step(true, true, TB, BEST, t, A, B, I2, I1);
                    step(true, true, TB, BEST, t + 1, B, A, I1, I2);
                }
                for (; t + 1 < te && t + 1 < tail_beg; t += 2) {
                    if (TB) {
                        step(false, false, true, false, t, A, B, I2, I1);
                        step(false, false, true, false, t + 1, B, A, I1, I2);
                    } else if (BEST && st == lastst) {
                        step(false, false, false, true, t, A, B, I2, I1);
                        step(false, false, false, true, t + 1, B, A, I1, I2);
                    } else {
                        step(false, false, false, false, t, A, B, I2, I1);
                        step(false, false, false, false, t + 1, B, A, I1, I2);
                    }
                }
                for (; t + 1 < te; t += 2) {
                    step(true, true, TB, BEST, t, A, B, I2, I1);
                    step(true, true, TB, BEST, t + 1, B, A, I1, I2);
                }
                if (t < te) { step(true, true, TB, BEST, t, A, B, I2, I1); ++t; }   // t1 odd: the sweep's end
            }
            if (seam_out) seam_flush(t, ts);
        };

        // ---------------------------------------------------- pass 1
        for (int s_ = 0; s_ < nstr; ++s_) {
            strip_init(s_);
            sweep(1, tend, false, true, true);
            wv_mem_sync();                            // seams written by every lane, read by the next strip
            // last row (:481-484): ">=" over the columns in visiting order
            // keeps the largest j among equal scores
            const int j0 = st * NWL_W + lane * K;
#pragma unroll
            for (int s = 0; s < K; ++s) {
                const int v = lrow[lane * K + s];
                if (j0 + s >= 1 && j0 + s < ylen && v >= bestR) { bestR = v; bestRj = j0 + s; }
            }
            wv_lds_sync();
        }
        // last column, rows [1, xlen - 1) (:481-484): ">=" in row order keeps the largest i
        for (int r = 1 + lane; r < xlen - 1; r += 64) {
            const int v = colbuf[(uint32_t)r * K + lasts];
            if (v >= bestC) { bestC = v; bestCi = r; }
        }
        // best cell (:481-484): last-row cells are visited after every other
        // row's, so they win ties; within each, ">=" kept the last visited
        red[lane * 4 + 0] = bestR; red[lane * 4 + 1] = bestRj; red[lane * 4 + 2] = bestC; red[lane * 4 + 3] = bestCi;
        wv_lds_sync();
        int bR = INT_MIN, bRj = 0, bC = INT_MIN, bCi = 0;
        for (int k = 0; k < 64; ++k) {
            const int *e = red + k * 4;
            if (e[0] > bR || (e[0] == bR && e[1] > bRj)) { bR = e[0]; bRj = e[1]; }
            if (e[2] > bC || (e[2] == bC && e[3] > bCi)) { bC = e[2]; bCi = e[3]; }
        }
        wv_lds_sync();
        int bscore, bx, by;
        if (bR >= bC) { bscore = bR; bx = xlen - 1; by = bRj; }
        else          { bscore = bC; bx = bCi; by = ylen - 1; }

        // ---------------------------------------------------- pass 2: the walk
        // the walk's state waits in LDS (every lane holds the same copy) while
        // a band is recomputed, so the sweep keeps its registers
        NwlWalk *ws = (NwlWalk *)red;
        *ws = NwlWalk{bx, by, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, false, false, false};
        int guard = 4 * (xlen + ylen) + 64, nband = 0;
        NwlBand bd = {tbw, X4, Y, -1, 0, 0};
        for (;;) {
            wv_lds_sync();
            NwlWalk w = *ws;
            nwl_walk_band(bd, w, lane, pscr, guard);
            if (!w.need) { *ws = w; break; }
            // recompute the band of strip need_j / NWL_W ending at the needed
            // cell's step, from the checkpoint below its first step
            const int s_ = w.need_j / NWL_W, lc = (w.need_j - s_ * NWL_W) / K, tc = w.need_i + lc;
            const int t1 = min(tc + 1, tend), m = max(t1 - band - 1, 0) / NWL_CK, t0 = 1 + m * NWL_CK;
            if (++nband > 4 * (nstr + (xlen + ylen) / 64 + 8)) { w.bad = true; *ws = w; break; }
            *ws = w;
            wv_lds_sync();
            strip_init(s_);
            seam_out = false;
            restore(m);
            bt0 = t0; tbb = tbw;
            sweep(t0, t1, true, false, false);
            wv_mem_sync();                            // band written by all lanes, read by the walkers
            bd.bst = s_; bd.bt0 = t0; bd.bt1 = t1;
        }
        wv_lds_sync();
        const NwlWalk w = *ws;
        if (w.run && !w.bad && lane == 0) pscr[w.nent - 1] = (IMSAME_MOVE_DIAG << 30) | (uint32_t)w.run;
        wv_mem_sync();
        // ---------------------------------------------------- result (nw_finish)
        bool acc = false;
        if (!w.bad)
            acc = (uint32_t)ylen < P.n_minlen && (uint32_t)w.len >= P.minlen[ylen] &&
                  (uint32_t)w.len < P.n_minident && (uint32_t)w.idn >= P.minident[w.len];
        if (w.bad && lane == 0) wv_atomic_or(P.flags, 2u);
        uint32_t poff = 0, plen = 0;
        if (acc && P.want_paths) {
            uint32_t off = 0;
            if (lane == 0) {
                off = wv_atomic_add(P.paths_used, (uint32_t)w.nent);
                if (off + (uint32_t)w.nent > P.paths_cap) { wv_atomic_or(P.flags, 1u); off = 0xFFFFFFFFu; }
            }
            off = wv_first(off);
            if (off != 0xFFFFFFFFu) {
                for (int k = lane; k < w.nent; k += 64) P.paths[off + k] = pscr[k];
                poff = off; plen = (uint32_t)w.nent;
            } else {                                  // arena full: the host re-walks this pair
                poff = 0xFFFFFFFFu; plen = (uint32_t)w.nent;
            }
        }
        if (lane == 0) {
            const int M = 2 * max(xlen, ylen);
            const int tail = w.px + w.py;             // one of them is 0
            imsame_read_result r;
            r.db_seq = sid; r.score = bscore; r.bx = (uint32_t)bx; r.by = (uint32_t)by;
            r.length = (uint32_t)w.len; r.identities = (uint32_t)w.idn;
            r.igaps = (uint32_t)w.ig; r.egaps = (uint32_t)w.eg;
            r.head_x = (uint32_t)(M - ((xlen - 1 - bx) + w.len + tail));
            r.head_y = (uint32_t)(M - ((ylen - 1 - by) + w.len + tail));
            r.ylen = (uint32_t)ylen; r.status = acc ? 1u : 2u;
            r.path_off = poff; r.path_len = plen;
            P.out[c] = r;
        }
        if (P.redo && lane == 0 && nband > nstr) wv_atomic_add(P.redo, (uint32_t)(nband - nstr));
        wv_mem_sync();
    }
}

__device__ void nwl_wave(const NwLaunch &P, uint8_t *wsm, const int lane, const uint32_t slot) {
    for (;;) {
        uint32_t c = 0;
        if (lane == 0) c = wv_atomic_add(P.counter, 1u);
        c = wv_first(c);
        if (c >= P.n_cand) break;
        nwl_cand(P, wsm, lane, slot, c);
    }
}

#ifndef IMSAME_WAVE_EMU
#ifndef NWL_WAVES_PER_EU
#define NWL_WAVES_PER_EU 3                 // 168 VGPRs: the sweeps' state without spills
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NWL_WAVES_PER_EU)))
void nwl_kernel(NwLaunch P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    const uint32_t slot = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + wib);   // wave-uniform
    nwl_wave(P, smem + wib * nwl_wave_lds(P.xstride), lane, slot);
}
#endif
