// nwp_kernel.hip -- IMSAME's NW + backtracking for LONG reads (longer than the
// short kernels' 160 columns) on PACKED PAIRS: two candidates per wave, one in
// each int16 half of every register, over nwl_kernel.hip's strips, seams,
// checkpoints and bands.  Included by imsame_dev.hip (and by
// tests/emu/wave_emu.cpp under IMSAME_WAVE_EMU) after nwl_kernel.hip.
//
// Reference: NW              alignmentFunctions.c:389-489
//            backtrackingNW  alignmentFunctions.c:493-560
//
// Why: the sweep is VALU-issue bound, and a packed op (v_pk_max_u16, v_perm,
// v_bitop3 on both halves) does the same cell of two candidates; the int32
// nwl_kernel issues 18.7 lane-instructions per cell, the packed short-read
// kernel 11.3 (profiles/nw_valu*.json).
//
// Mapping: nwl_kernel's -- strips of NWP_W = 640 columns, lane l owns NWP_K =
// 10 of them and walks the rows one lane behind its left neighbour (step t:
// row i = t - l); row state crosses lanes by DPP wave_shr:1 and strips by a
// seam; pass 1 keeps checkpoints every NWL_CK steps and the best cells, pass 2
// recomputes (strip, step) bands with traceback for backtrackingNW's walk.
// The cell recurrence is nw16_kernel.hip's (DP values biased by 2^15, gap
// terms as drifting state, decisions as packed signs), with two changes for
// range: the traceback signs compare against the maxima the cell computes
// anyway (d0 - max(d0, lu), l0 - lu), so a gap term far below the row's T
// cannot wrap them.
//
// Range.  A 10 kbp x 12 kbp matrix holds scores up to ~4e4: no one int16
// frame holds them.  Each LANE keeps each half relative to its own frame
// off[h] (int32), moved every 64-step block to the lane's current T (B[0]);
// the left neighbour's row state (T, mf, l0) is shifted into this lane's frame
// as it arrives (dl = off(left) - off(own), one v_pk_add per value per step),
// and seams hold absolute int32.  The reference's recurrence is not smooth --
// an up or left term decays from the FIRST maximum of its column or row, so
// neighbouring cells can differ by thousands -- so nothing is assumed about
// the spread: every block start reduces the wave's absolute extremes per half
// (T, gap terms u0 / l0, maxima mcS / mf, and the seam rows of the block) and
// bounds every compared difference of the block by them (every frame is one
// of the wave's T; within a block a T moves <= 4 per step and a gap term falls
// <= 64 |eg|):
//     maxima - T  <= (Mmax - Tmin) + (Tmax - Tmin) + NWP_G + 7
//     T - gap     <= (Tmax - Gmin) + (Tmax - Tmin) + NWP_G + 64|eg| + 20
// A wave whose bound reaches 2^15 abandons its pair before that block and runs
// both candidates through nwl_cand (int32) instead -- same results, counted
// in NwLaunch::fbk.  The traceback signs compare against the maxima the cell
// computes anyway (d0 - max(d0, lu), l0 - lu), which the second bound covers.
// nwp_fits only keeps launches that are likely to pass (records up to ~14 kbp
// at the default gaps: the drift |eg| (L + 64) plus a budget for the spread).
//
// Column 0 (lane 0 of strip 0) keeps frame 0: its T is s(x, y) and its
// neighbours' within +-4 per column, and the sentinels of column 1 (mc[0]
// never updated, mf = -inf) stay put.

#ifndef NWP_K
#define NWP_K    10                       // columns per lane
#endif
#define NWP_W    (64 * NWP_K)             // columns per strip
#define NWP_NST  (4 * NWP_K + 7)          // A, B, mcS, u0 per column; I1, I2, outT, outMS, outL; off[2]
#define NWP_NREC nw16_nrec(NWP_K)         // traceback dwords per lane per step (TbWords<NWP_K>)
#define NWP_G    (4 * 64 + 64)            // how far a T moves within a 64-step block (+4 per step; column 0: +-44)
#define NWP_S2   2308                     // nwp_fits: the T spread it budgets

#ifdef IMSAME_WAVE_EMU
// Emulator only: the block-start bound above is a proof about the steps
// inside a block; the emulator checks its conclusion at every step.  Each
// packed operation whose result a live cell uses (rows [1, xlen), columns
// [1, ylen) of that half) is checked for int16 wrap in that half:
// tests/emu/wave_emu.cpp counts the violations (emu_nwp_range_violations).
extern std::atomic<uint64_t> g_nwp_viol;
static inline void nwp_chk(unsigned live, int kind, uint32_t a, uint32_t b) {
    for (int h = 0; h < 2; ++h) {
        if (!(live >> h & 1u)) continue;
        const int ua = (int)(h ? a >> 16 : a & 0xFFFFu), ub = (int)(h ? b >> 16 : b & 0xFFFFu);
        bool bad;
        if (kind == 0) { const int s = ua + (int)(int16_t)ub; bad = s < 0 || s > 0xFFFF; }   // pk_add, b signed
        else if (kind == 1) { const int d = ua - ub; bad = d < -32768 || d > 32767; }        // pk_sub -> sign
        else bad = ua < ub;                                                                  // biased decrement
        if (bad) g_nwp_viol.fetch_add(1, std::memory_order_relaxed);
    }
}
#define NWP_CHK(live, kind, a, b) nwp_chk(live, kind, a, b)
#else
#define NWP_CHK(live, kind, a, b) ((void)0)
#endif

// |ig| + |eg| (L + 64): the drift bound of the launch (NwLaunch::rlim)
__host__ static inline int64_t nwp_rlim(int64_t ig, int64_t eg, uint64_t xcap, uint64_t ymax) {
    return -ig + -eg * (int64_t)(std::max<uint64_t>(xcap, ymax) + 64);
}
// is the launch likely to fit the packed long kernel?  (nwl_fits, and the range
// above with a budget of NWP_S2 for the T spread)
__host__ static inline bool nwp_fits(int64_t ig, int64_t eg, uint64_t xcap, uint64_t ymax) {
    if (!nwl_fits(ig, eg, ymax) || -ig > 1024 || -eg > 16) return false;
    return 2 * NWP_S2 + nwp_rlim(ig, eg, xcap, ymax) + 16 + 100 <= 32767;
}
// Launch shape: NWP_W-column strips, the two records two rows per byte.  A
// wave that falls back runs nwl_cand in the same slot and LDS, so every size
// below is also at least nwl_kernel's (its strips are NWL_W wide).
__host__ static inline NwShape nwp_shape(uint32_t ymax, uint32_t xcap) {
    NwShape s = nwl_shape(ymax, xcap);
    s.nstr = std::max(1, (int)((ymax + NWP_W - 1) / NWP_W));
    s.xstride = std::max(s.xstride, ((s.xcap + 1) / 2 + 16 + 15) & ~15);
    return s;
}
__host__ static inline uint64_t nwp_ck_words(const NwShape &s, uint32_t ymax) {
    return std::max<uint64_t>((uint64_t)s.nstr * nwl_ncks(s.steps) * NWP_NST * 64, nwl_ck_words(nwl_shape(ymax, s.xcap)));
}
// seams: six planes per strip (T, mf score, l0 of each half, absolute)
__host__ static inline uint64_t nwp_seam_words(const NwShape &s, uint32_t ymax) {
    return std::max<uint64_t>((uint64_t)s.nstr * (s.xcap + 1) * 6, nwl_seam_words(nwl_shape(ymax, s.xcap)));
}
__host__ __device__ static inline uint64_t nwp_band_words() { return (uint64_t)(NWL_BAND + NWL_CK + 64) * 64 * NWP_NREC; }
// pass 1: each half's last-column records (NWP_K packed cells + the two frame
// offsets per row); pass 2: the band + a path scratch per half; and whatever
// nwl_cand needs
__host__ static inline uint64_t nwp_tb_words(const NwShape &s, uint32_t ymax) {
    const uint64_t p1 = (uint64_t)2 * s.xcap * (NWP_K + 2) + 64;
    const uint64_t p2 = nwp_band_words() + 2 * ((uint64_t)s.xcap + ymax + 64 + 1);
    return std::max(std::max(p1, p2), nwl_tb_words(nwl_shape(ymax, s.xcap), ymax));
}

// 2-bit code of row i of half h (two rows per byte: A bits 0-1 / 4-5, B 2-3 / 6-7)
WV_DEVICE uint32_t nwp_code(const uint8_t *X2, int i, int h) { return (X2[i >> 1] >> (4 * (i & 1) + 2 * h)) & 3u; }

// one lane's view of the packed band for half h: strip bst, steps [bt0, bt1)
struct NwpBand {
    const uint32_t *tb; const uint8_t *X2; const uint8_t *Y;
    int h, bst, bt0, bt1;
    __device__ bool has(int i, int j) const {
        const int st = j / NWP_W, l = (j - st * NWP_W) / NWP_K, t = i + l;
        return st == bst && t >= bt0 && t < bt1;
    }
    __device__ uint32_t nib(int i, int j) const {
        const int jj = j - bst * NWP_W, l = jj / NWP_K, s = jj - l * NWP_K, t = i + l;
        return tb16_nib<NWP_K>(tb + ((uint32_t)(t - bt0) * 64u + (uint32_t)l) * NWP_NREC, s, h);
    }
    __device__ bool match(int i, int j) const { return nwp_code(X2, i, h) == base_code(Y[j]); }
};

__device__ void nwp_wave(const NwLaunch &P, uint8_t *wsm, const int lane, const uint32_t slot) {
    constexpr int K = NWP_K;
    const int ig = P.igap, eg = P.egap;
    const uint32_t H = NW16_H, NBIG = pk1(-NW16_BIG) ^ NW16_H, PBIG = pk1(NW16_BIG) ^ NW16_H;
    const uint32_t EGN = pk1(-eg), IGEN = pk1(-(ig + eg));      // gap magnitudes (biased subtracts)
    const int64_t LIM = P.nwp_s > 0 ? P.nwp_s : 32767 - 16;     // tests: a tiny limit forces the fallback
    const int DEC = 64 * -eg + 16;                                // a gap term's fall within a block
    uint8_t *X2 = wsm;
    int *red = (int *)(wsm + P.xstride);                          // 64 lanes x 8 ints, then the walks
    uint32_t *tbw = P.tb + (uint64_t)slot * P.tb_wave_dw;
    int *seam = P.bnd + (uint64_t)slot * P.bnd_wave;
    uint32_t *ckw = P.ck + (uint64_t)slot * P.ck_wave_dw + lane;
    const int ncks = nwl_ncks(P.steps);
    const int band = (P.band_w > 0 && P.band_w < NWL_BAND) ? P.band_w : NWL_BAND;
    const uint64_t pstride = (uint64_t)P.xcap + P.n_minlen + 64;   // path scratch per half (n_minlen = ymax + 1)
    for (;;) {
        uint32_t base = 0;
        if (lane == 0) base = wv_atomic_add(P.counter, 2u);
        base = wv_first(base);
        if (base >= P.n_cand) break;
        // the pair: an absent B repeats A (computed, never written)
        const bool valid[2] = {true, base + 1 < P.n_cand};
        const uint32_t cidx[2] = {base, valid[1] ? base + 1 : base};
        uint32_t sid[2];
        int xl[2], yl[2];
        const uint8_t *Xg[2], *Yp[2];
        for (int h = 0; h < 2; ++h) {
            const uint32_t rd = P.cand_read[cidx[h]];
            sid[h] = P.cand_sid[cidx[h]];
            const uint64_t xo = P.db_start[sid[h]];
            xl[h] = (int)(P.db_start[sid[h] + 1] - xo); Xg[h] = P.db + xo;
            const uint64_t yo = P.q_start[rd];
            yl[h] = (int)(P.q_start[rd + 1] - yo); Yp[h] = P.q + yo;
        }
        const int xmax = max(xl[0], xl[1]), xmin = min(xl[0], xl[1]), ymx = max(yl[0], yl[1]);
        // both records in LDS, two rows per byte; rows past a record repeat its
        // last base (the lockstep garbage of the shorter one stays a DP)
        for (int b = lane; b < (xmax + 1) / 2; b += 64) {
            uint32_t v = 0;
#pragma unroll
            for (int k = 0; k < 2; ++k)
                for (int h = 0; h < 2; ++h)
                    v |= base_code(Xg[h][min(2 * b + k, max(xl[h] - 1, 0))]) << (4 * k + 2 * h);
            X2[b] = (uint8_t)v;
        }
        wv_lds_sync();
        const int nstr = (ymx + NWP_W - 1) / NWP_W;
        const int tend = xmax - 1 + 64;               // the last lane's last row at step tend - 1
        const int SP = xmax + 1;                      // seam plane stride: rows 0..xmax
        int lastst[2], lastl[2], lasts[2];
        for (int h = 0; h < 2; ++h) {
            lastst[h] = (yl[h] - 1) / NWP_W;
            lastl[h] = ((yl[h] - 1) - lastst[h] * NWP_W) / K;
            lasts[h] = (yl[h] - 1) - lastst[h] * NWP_W - lastl[h] * K;
        }
        uint32_t *cb[2] = {tbw, tbw + (uint64_t)P.xcap * (K + 2)};   // last-column records, row r at r * (K + 2)
        int bestR[2] = {INT_MIN, INT_MIN}, bestRj[2] = {0, 0};

        // ---- state of one strip's sweep, shared by both passes
        uint32_t yreg[K], A[K], B[K], dI[K], mcS[K], u0[K];
        uint32_t I1 = 0, I2 = 0, outT = 0, outMS = 0, outL = 0;
        int off[2] = {0, 0};                          // this lane's frame per half
        uint32_t dl = 0;                              // left neighbour's frame - own (lane 0: 0)
        // row selectors: xs = this lane's row ([xA, xA, xB, xB] bytes), xq =
        // the block's rows (lane l = row t_b + l, popped by the lead lane)
        uint32_t xs = 0, xq = 0;
        // the previous strip's right edge in lane 0's frame (R: this block's
        // rows, lane l = row t_b + l), N the next block's (absolute, in
        // flight); W collects the last lane's edge, flushed every block
        uint32_t R0 = 0, R1 = 0, R2 = 0, W0 = 0, W1 = 0, W2 = 0;
        int N[6] = {0, 0, 0, 0, 0, 0};
        int st = 0;
        bool leadc0 = false, seam_in = false, seam_out = false;
        const int *seam_rd = seam;
        int *seam_wr = seam;
        uint32_t *tbb = tbw;
        int bt0 = 0;
        auto xsel_row = [&](int r) {
            r = min(max(r, 0), xmax - 1);
            const uint32_t b = (X2[r >> 1] >> (4 * (r & 1))) & 0xFu;
            return wv_perm(b >> 2, b & 3u, 0x04040000u);
        };
        auto seam_load = [&](const int r0) {          // edge rows r0 + lane (clamped into [1, xmax))
            const int r = min(max(r0 + lane, 1), max(xmax - 1, 1));
#pragma unroll
            for (int p = 0; p < 6; ++p) N[p] = seam_rd[p * SP + r];
        };
        // N -> R in lane 0's (new) frame (rebase() counted the rows in the wave's extremes)
        auto seam_take = [&]() {
            const int oa = wv_readlane(off[0], 0), ob = wv_readlane(off[1], 0);
            R0 = pk2(N[0] - oa, N[1] - ob) ^ H; R1 = pk2(N[2] - oa, N[3] - ob) ^ H; R2 = pk2(N[4] - oa, N[5] - ob) ^ H;
        };
        // W = steps [t - 64, t) of the last lane: lane l row t - 127 + l.  Only
        // the rows of the block that began at step tb (its frame: the last
        // lane's, not yet moved); after a partial last block the lanes below
        // hold rows the previous flush wrote, in the previous frame
        auto seam_flush = [&](const int t, const int tb) {
            const int oa = wv_readlane(off[0], 63), ob = wv_readlane(off[1], 63);
            const int r = t - 127 + lane;
            if (r >= 1 && r < xmax && r >= tb - 63) {
                seam_wr[r] = pk_score(W0, 0) + oa;          seam_wr[SP + r] = pk_score(W0, 1) + ob;
                seam_wr[2 * SP + r] = pk_score(W1, 0) + oa; seam_wr[3 * SP + r] = pk_score(W1, 1) + ob;
                seam_wr[4 * SP + r] = pk_score(W2, 0) + oa; seam_wr[5 * SP + r] = pk_score(W2, 1) + ob;
            }
        };
        // strip setup: y codes, row 0 (:404-413), frames at 0
        auto strip_init = [&](const int s_) {
            st = s_;
            const int j0 = st * NWP_W + lane * K;
            leadc0 = st == 0 && lane == 0;
            seam_in = st > 0;
            seam_out = st + 1 < nstr;
            seam_rd = seam + (uint64_t)(st > 0 ? st - 1 : 0) * 6 * SP;
            seam_wr = seam + (uint64_t)st * 6 * SP;
            const uint32_t xs0 = xsel_row(0);
#pragma unroll
            for (int s = 0; s < K; ++s) {
                const int j = j0 + s;
                const uint32_t ya = j < yl[0] ? base_code(Yp[0][j]) : 0u, yb = j < yl[1] ? base_code(Yp[1][j]) : 0u;
                yreg[s] = ya | ((ya | 4u) << 8) | (yb << 16) | ((yb | 4u) << 24);
                A[s] = wv_perm(NW16_TBL_HI, NW16_TBL_LO, xs0 ^ yreg[s]) ^ H;
                B[s] = A[s];
            }
            uint32_t yprev = 0;
            if (j0 > 0) {
                const uint32_t ya = base_code(Yp[0][min(j0 - 1, yl[0] - 1)]), yb = base_code(Yp[1][min(j0 - 1, yl[1] - 1)]);
                yprev = ya | ((ya | 4u) << 8) | (yb << 16) | ((yb | 4u) << 24);
            }
            const uint32_t t0prev = wv_perm(NW16_TBL_HI, NW16_TBL_LO, xs0 ^ yprev) ^ H;
#pragma unroll
            for (int s = 0; s < K; ++s) {
                // mc[j-1] = (T[0][j-1], row 0); row 0 stands in for rows -1 and -2
                dI[s] = ((s == 0) ? t0prev : A[s - 1]) - IGEN;
                mcS[s] = dI[s];
                u0[s] = dI[s];
                if (j0 + s == 1) mcS[s] = PBIG;                 // mc[0] is never updated (:476)
            }
            I1 = t0prev; I2 = t0prev;
            outT = A[K - 1]; outMS = H; outL = H;
            off[0] = off[1] = 0; dl = 0;
        };
        // one step (roles (cur, own) swap every step): HEAD = some lane may be
        // at row <= 1; CAREFUL = rows may be a record's last (or past it); TB =
        // write the traceback words (pass 2, band step t - bt0); BEST = pass 1:
        // last row (CAREFUL steps) and last column records (the last strips)
        auto step = [&](const bool HEAD, const bool CAREFUL, const bool TB, const bool BEST, const int t,
                        uint32_t (&cur)[K], const uint32_t (&own)[K], uint32_t &in0, const uint32_t in1) {
            // row state from the left neighbour, into this lane's frame (lane 0:
            // the previous strip's edge, already in it; strip 0: unused)
            const uint32_t R0n = (uint32_t)wv_shl1((int)R0), R1n = (uint32_t)wv_shl1((int)R1),
                           R2n = (uint32_t)wv_shl1((int)R2);
            const uint32_t sN = pk_add((uint32_t)wv_shr1_fill((int)outT, (int)R0), dl);
            const uint32_t mS = pk_add((uint32_t)wv_shr1_fill((int)outMS, (int)R1), dl);
            const uint32_t mL0 = pk_add((uint32_t)wv_shr1_fill((int)outL, (int)R2), dl);
#ifdef IMSAME_WAVE_EMU
            // the halves whose cell (i, j0 + s) is live
            auto live = [&](int s) {
                unsigned m = 0;
                for (int h = 0; h < 2; ++h) {
                    const int j = st * NWP_W + lane * K + s;
                    const int ii = t - lane;
                    m |= (unsigned)(ii >= 1 && ii < xl[h] && j >= 1 && j < yl[h]) << h;
                }
                return m;
            };
            {   // (the exchanges are lock-step: every lane makes them)
                const uint32_t sT = (uint32_t)wv_shr1_fill((int)outT, (int)R0),
                               sM = (uint32_t)wv_shr1_fill((int)outMS, (int)R1),
                               sL = (uint32_t)wv_shr1_fill((int)outL, (int)R2);
                const unsigned l0m = live(0), l1m = (st == 0 && lane == 1) ? 0u : l0m;  // column 1: column 0's sentinels
                NWP_CHK(l0m, 0, sT, dl); NWP_CHK(l1m, 0, sM, dl); NWP_CHK(l1m, 0, sL, dl);
            }
#endif
            R0 = R0n; R1 = R1n; R2 = R2n;
            const uint32_t xqn = (uint32_t)wv_shl1((int)xq);
            xs = (uint32_t)wv_shr1_fill((int)xs, (int)xq);
            xq = xqn;
            const int i = t - lane;
            const bool pre = HEAD && i < 1;
            const bool row1 = HEAD && i <= 1;         // up invalid, mc frozen (:449, :476)
            uint32_t mfS = mS, l0 = mL0;
            TbWords<K> tw = {};
#pragma unroll
            for (int s = 0; s < K; ++s) {
                const uint32_t d0 = (s == 0) ? in1 : own[s - 1];     // T[i-1][j-1]
                const uint32_t tl = (s == 0) ? sN : cur[s - 1];      // T[i][j-1]
                const uint32_t sc = wv_perm(NW16_TBL_HI, NW16_TBL_LO, xs ^ yreg[s]);
                const uint32_t up = row1 ? NBIG : u0[s];
                const uint32_t lu = pk_maxu(l0, up), m = pk_maxu(d0, lu);
#ifdef IMSAME_WAVE_EMU
                {
                    const unsigned lv = live(s), lv2 = (i >= 2) ? lv : 0u;
                    NWP_CHK(lv, 0, m, sc);
                    if (TB) { NWP_CHK(lv, 1, l0, lu); NWP_CHK(lv, 1, d0, m); }
                    NWP_CHK(lv2, 1, mcS[s], dI[s]);
                    NWP_CHK(lv2, 2, wv_bfi(pk_neg_mask(pk_sub(mcS[s], dI[s])), dI[s], u0[s]), EGN);
                    NWP_CHK(lv, 1, tl, mfS);
                    NWP_CHK(lv, 2, d0, IGEN);
                    if (!(s == 0 && leadc0)) NWP_CHK(lv, 2, l0, EGN);
                }
#endif
                uint32_t v = pk_add(m, sc);
                if (s == 0 && leadc0) v = sc ^ H;                        // column 0 (:426)
                cur[s] = pre ? own[s] : v;
                // move bits (:457-472): not diagonal = m > d0, up > left = lu > l0
                // (differences to the maxima: no wrap whatever the losing term)
                const uint32_t P2 = TB ? wv_perm(pk_sub(l0, lu), pk_sub(d0, m), 0x0B0A0908u) : 0u;
                // column max of column j-1 over rows <= i-2, strict > (:476-480), in
                // the +ig+eg frame: dI[s] = T[i-2][j-1] + ig + eg
                const uint32_t mU = pk_neg_mask(pk_sub(mcS[s], dI[s]));
                const uint32_t u0n = wv_bfi(mU, dI[s], u0[s]) - EGN;
                u0[s] = row1 ? u0[s] : u0n;
                mcS[s] = wv_bfi(mU, dI[s], mcS[s]);
                // row state for column j+1: tested on row i, taken from row i-1 (:434-438)
                const uint32_t mnL = pk_neg_mask(pk_sub(tl, mfS));     // 0xFFFF: mf kept (not L)
                dI[s] = d0 - IGEN;                                      // the next row's
                l0 = wv_bfi(mnL, l0 - EGN, dI[s]);
                mfS = wv_bfi(mnL, mfS, d0);
                if (s == 0 && leadc0) { mfS = NBIG; l0 = NBIG; }          // j = 1: no left move
                if (TB) tw.add(s, P2, mU, mnL);
            }
            if (TB) tw.store(tbb + ((uint32_t)(t - bt0) * 64u + (uint32_t)lane) * NWP_NREC);
            if (BEST) {
                const int j0 = st * NWP_W + lane * K;
                for (int h = 0; h < 2; ++h) {
                    // last row (:481-484): ">=" in visiting order keeps the largest j
                    if (CAREFUL && i >= 1 && i == xl[h] - 1) {
#pragma unroll
                        for (int s = 0; s < K; ++s) {
                            const int v = pk_score(cur[s], h) + off[h];
                            if (j0 + s >= 1 && j0 + s < yl[h] && v >= bestR[h]) { bestR[h] = v; bestRj[h] = j0 + s; }
                        }
                    }
                    // last column, rows [1, xlen - 1): the owner lane's cells and frame
                    if (st == lastst[h] && lane == lastl[h] && i >= 1 && i < xl[h] - 1) {
                        uint32_t *q = cb[h] + (uint32_t)i * (K + 2);
#pragma unroll
                        for (int s = 0; s < K; ++s) q[s] = cur[s];
                        q[K] = (uint32_t)off[0]; q[K + 1] = (uint32_t)off[1];
                    }
                }
            }
            if (seam_out) {                           // the last lane's edge, row i, into W
                W0 = (uint32_t)wv_shl1_fill((int)W0, (int)cur[K - 1]);
                W1 = (uint32_t)wv_shl1_fill((int)W1, (int)mfS);
                W2 = (uint32_t)wv_shl1_fill((int)W2, (int)l0);
            }
            in0 = pre ? in1 : sN;
            outT = cur[K - 1]; outMS = mfS; outL = l0;
        };
        // checkpoint m of strip st: the state before step 1 + m*NWL_CK (a block
        // start, before its rebase), roles (A, B), (I2, I1); dI follows from A and
        // I2 (nw16_kernel.hip: save())
        auto save = [&](const int m) {
            uint32_t *p = ckw + (uint32_t)((st * ncks + m) * NWP_NST) * 64u;
#pragma unroll
            for (int s = 0; s < K; ++s) {
                p[s * 64] = A[s]; p[(K + s) * 64] = B[s];
                p[(2 * K + s) * 64] = mcS[s]; p[(3 * K + s) * 64] = u0[s];
            }
            p[4 * K * 64] = I1; p[(4 * K + 1) * 64] = I2;
            p[(4 * K + 2) * 64] = outT; p[(4 * K + 3) * 64] = outMS; p[(4 * K + 4) * 64] = outL;
            p[(4 * K + 5) * 64] = (uint32_t)off[0]; p[(4 * K + 6) * 64] = (uint32_t)off[1];
        };
        auto restore = [&](const int m) {
            const uint32_t *p = ckw + (uint32_t)((st * ncks + m) * NWP_NST) * 64u;
#pragma unroll
            for (int s = 0; s < K; ++s) {
                A[s] = p[s * 64]; B[s] = p[(K + s) * 64];
                mcS[s] = p[(2 * K + s) * 64]; u0[s] = p[(3 * K + s) * 64];
            }
            I1 = p[4 * K * 64]; I2 = p[(4 * K + 1) * 64];
            outT = p[(4 * K + 2) * 64]; outMS = p[(4 * K + 3) * 64]; outL = p[(4 * K + 4) * 64];
            off[0] = (int)p[(4 * K + 5) * 64]; off[1] = (int)p[(4 * K + 6) * 64];
#pragma unroll
            for (int s = 0; s < K; ++s) dI[s] = (s ? A[s - 1] : I2) - IGEN;
        };
        // block start: move the frame to the lane's T (B[0], its last row) and
        // check the ranges; true if any value is outside them
        auto rebase = [&](const int t) {
            const uint32_t D = leadc0 ? 0u : (B[0] ^ H);
            off[0] += (int)(int16_t)(D & 0xFFFFu); off[1] += (int)(int16_t)(D >> 16);
            uint32_t hi = 0, lo = 0xFFFFFFFFu, glo = 0xFFFFFFFFu, mhi = 0;
#pragma unroll
            for (int s = 0; s < K; ++s) {
                A[s] = pk_sub(A[s], D); B[s] = pk_sub(B[s], D); dI[s] = pk_sub(dI[s], D);
                mcS[s] = pk_sub(mcS[s], D); u0[s] = pk_sub(u0[s], D);
                hi = pk_maxu(hi, pk_maxu(A[s], B[s])); lo = pk_minu(lo, pk_minu(A[s], B[s]));
                // column 0's lane: slot 0's column state belongs to column -1
                // (never read) and slot 1 holds column 1's sentinel
                glo = pk_minu(glo, (s == 0 && leadc0) ? H : u0[s]);
                mhi = pk_maxu(mhi, (s <= 1 && leadc0) ? H : mcS[s]);
            }
            I1 = pk_sub(I1, D); I2 = pk_sub(I2, D);
            outT = pk_sub(outT, D); outMS = pk_sub(outMS, D); outL = pk_sub(outL, D);
            const uint32_t i12hi = leadc0 ? H : pk_maxu(I1, I2), i12lo = leadc0 ? H : pk_minu(I1, I2);   // (column -1)
            hi = pk_maxu(hi, pk_maxu(i12hi, outT)); lo = pk_minu(lo, pk_minu(i12lo, outT));
            glo = pk_minu(glo, outL); mhi = pk_maxu(mhi, outMS);
            const int la = wv_shr1(off[0]), lb = wv_shr1(off[1]);
            dl = lane ? pk2(la - off[0], lb - off[1]) : 0u;
            // the wave's extremes, absolute, per half: T, gap terms, maxima (and
            // the seam rows lane 0 takes in this block)
            int ex[2][4];                              // T max, -T min, -gap min, max-term max
            for (int h = 0; h < 2; ++h) {
                ex[h][0] = pk_score(hi, h) + off[h]; ex[h][1] = -(pk_score(lo, h) + off[h]);
                ex[h][2] = -(pk_score(glo, h) + off[h]); ex[h][3] = pk_score(mhi, h) + off[h];
                if (seam_in && t + lane < xmax) {
                    ex[h][0] = max(ex[h][0], N[h]); ex[h][1] = max(ex[h][1], -N[h]);
                    ex[h][2] = max(ex[h][2], -N[4 + h]); ex[h][3] = max(ex[h][3], N[2 + h]);
                }
            }
            for (int o = 32; o > 0; o >>= 1)
                for (int h = 0; h < 2; ++h)
                    for (int k = 0; k < 4; ++k) ex[h][k] = max(ex[h][k], wv_shfl_xor(ex[h][k], o));
            // every lane's frame is one of the wave's T, so within a block (T
            // moves <= G per step and crosses lanes exactly; gap terms fall
            // <= DEC) the compared differences are bounded by
            //   maxima - T  <= (Mmax - Tmin) + span + G + 7
            //   T - gap     <= (Tmax - Gmin) + span + G + DEC + 4
            // (span = Tmax - Tmin); both must stay below 2^15
            bool bad = false;
            for (int h = 0; h < 2; ++h) {
                const int64_t span = (int64_t)ex[h][0] + ex[h][1];
                bad = bad || (int64_t)ex[h][3] + ex[h][1] + span + NWP_G + 7 > LIM ||
                      (int64_t)ex[h][0] + ex[h][2] + span + NWP_G + DEC + 4 > LIM;
            }
#ifdef IMSAME_WAVE_EMU
            if (bad && lane == 0 && getenv("IMSAME_NWP_DEBUG"))
                fprintf(stderr, "[nwp] st %d t %d: T [%d, %d] gap >= %d max <= %d | B: T [%d, %d] gap >= %d max <= %d\n",
                        st, t, -ex[0][1], ex[0][0], -ex[0][2], ex[0][3], -ex[1][1], ex[1][0], -ex[1][2], ex[1][3]);
#endif
            return bad;
        };
        // run steps [ts, t1) from the state before step ts (ts = 1 mod NWL_CK)
        // in blocks of 64 steps; true if a block start found a value out of range
        auto sweep = [&](const int ts, const int t1, const bool TB, const bool CKS) {
            const bool BEST = !TB, lastsw = BEST && (st == lastst[0] || st == lastst[1]);
            xs = xsel_row(ts - 1 - lane);             // as the left neighbour would hand it over
            if (seam_in) seam_load(ts);
            const int head_end = 66, tail_beg = xmin - 2;          // fast steps: every lane in rows [2, xmin - 1)
            int t = ts, tb = ts;                      // tb: the current block's first step
            while (t < t1) {
                if (seam_out && t > ts) seam_flush(t, tb);
                tb = t;
                if (CKS && (t - 1) % NWL_CK == 0) save((t - 1) / NWL_CK);
                bool bad = rebase(t);
                if (seam_in) { seam_take(); seam_load(t + 64); }
                xq = xsel_row(t + lane);
                if (wv_any(bad)) return true;
                const int te = min(t + 64, t1);
                for (; t + 1 < te && t + 1 < head_end; t += 2) {
                    step(true, true, TB, BEST, t, A, B, I2, I1);
                    step(true, true, TB, BEST, t + 1, B, A, I1, I2);
                }
                for (; t + 1 < te && t + 1 < tail_beg; t += 2) {
                    if (TB) {
                        step(false, false, true, false, t, A, B, I2, I1);
                        step(false, false, true, false, t + 1, B, A, I1, I2);
                    } else if (lastsw) {
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
            if (seam_out) seam_flush(t, tb);
            return false;
        };

        // ---------------------------------------------------- pass 1
        bool ovf = false;
        for (int s_ = 0; s_ < nstr && !ovf; ++s_) {
            strip_init(s_);
            ovf = sweep(1, tend, false, true);
            wv_mem_sync();                            // seams / last-column records, read by other lanes
        }
        NwlWalk *wsp = (NwlWalk *)red;                // pass 2's walk state per half (after the reduction)
        int bscore[2] = {0, 0}, bx[2] = {0, 0}, by[2] = {0, 0};
        if (!ovf) {
            // last column, rows [1, xlen - 1) (:481-484): ">=" in row order keeps the largest i
            int bestC[2] = {INT_MIN, INT_MIN}, bestCi[2] = {0, 0};
            for (int h = 0; h < 2; ++h)
                for (int r = 1 + lane; r < xl[h] - 1; r += 64) {
                    const uint32_t *q = cb[h] + (uint32_t)r * (K + 2);
                    const int v = pk_score(q[lasts[h]], h) + (int)q[K + h];
                    if (v >= bestC[h]) { bestC[h] = v; bestCi[h] = r; }
                }
            // best cell (:481-484): last-row cells are visited after every other
            // row's, so they win ties; within each, ">=" kept the last visited
            for (int h = 0; h < 2; ++h) {
                red[lane * 8 + 4 * h + 0] = bestR[h]; red[lane * 8 + 4 * h + 1] = bestRj[h];
                red[lane * 8 + 4 * h + 2] = bestC[h]; red[lane * 8 + 4 * h + 3] = bestCi[h];
            }
            wv_lds_sync();
            for (int h = 0; h < 2; ++h) {
                int bR = INT_MIN, bRj = 0, bC = INT_MIN, bCi = 0;
                for (int k = 0; k < 64; ++k) {
                    const int *e = red + k * 8 + 4 * h;
                    if (e[0] > bR || (e[0] == bR && e[1] > bRj)) { bR = e[0]; bRj = e[1]; }
                    if (e[2] > bC || (e[2] == bC && e[3] > bCi)) { bC = e[2]; bCi = e[3]; }
                }
                if (bR >= bC) { bscore[h] = bR; bx[h] = xl[h] - 1; by[h] = bRj; }
                else          { bscore[h] = bC; bx[h] = bCi; by[h] = yl[h] - 1; }
            }
            wv_lds_sync();

            // ------------------------------------------------ pass 2: the walks
            // each half walks the current band until it needs a cell outside it;
            // the first half that does gets the next band (both halves' bits)
            for (int h = 0; h < 2; ++h) {
                wsp[h] = NwlWalk{bx[h], by[h], 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, false, !valid[h], false};
            }
            int guard[2] = {4 * (xl[0] + yl[0]) + 64, 4 * (xl[1] + yl[1]) + 64}, nband = 0;
            int bst = -1, bb0 = 0, bb1 = 0;
            const int maxband = 4 * (2 * nstr + (xmax + ymx) / 32 + 16);
            for (;;) {
                int hn = -1, ni = 0, nj = 0;
                for (int h = 0; h < 2; ++h) {
                    wv_lds_sync();
                    NwlWalk w = wsp[h];
                    if (!w.done && !w.bad) {
                        const NwpBand bd = {tbw, X2, Yp[h], h, bst, bb0, bb1};
                        nwl_walk_band(bd, w, lane, tbw + nwp_band_words() + h * pstride, guard[h]);
                    }
                    wv_lds_sync();
                    wsp[h] = w;
                    if (w.need && hn < 0) { hn = h; ni = w.need_i; nj = w.need_j; }
                }
                if (hn < 0) break;
                // recompute the band of strip nj / NWP_W ending at the needed
                // cell's step, from the checkpoint below its first step
                const int s_ = nj / NWP_W, lc = (nj - s_ * NWP_W) / K, tc = ni + lc;
                const int t1 = min(tc + 1, tend), m = max(t1 - band - 1, 0) / NWL_CK, t0 = 1 + m * NWL_CK;
                if (++nband > maxband) {
                    wv_lds_sync();
                    for (int h = 0; h < 2; ++h) if (wsp[h].need) { NwlWalk w = wsp[h]; w.bad = true; wsp[h] = w; }
                    break;
                }
                strip_init(s_);
                seam_out = false;
                restore(m);
                bt0 = t0; tbb = tbw;
                if (sweep(t0, t1, true, false)) { ovf = true; break; }
                wv_mem_sync();                        // band written by all lanes, read by the walkers
                bst = s_; bb0 = t0; bb1 = t1;
            }
            wv_lds_sync();
            if (!ovf && P.redo && lane == 0 && nband > 2 * nstr) wv_atomic_add(P.redo, (uint32_t)(nband - 2 * nstr));
        }
        if (ovf) {
            // a value left the proof's range: both candidates through the int32 kernel
            if (lane == 0 && P.fbk) wv_atomic_add(P.fbk, 1u);
            wv_mem_sync();
            for (int h = 0; h < 2; ++h)
                if (valid[h]) nwl_cand(P, wsm, lane, slot, cidx[h]);
            continue;
        }
        // ---------------------------------------------------- results (nw_finish)
        for (int h = 0; h < 2; ++h) {
            const NwlWalk w = wsp[h];
            uint32_t *pscr = tbw + nwp_band_words() + h * pstride;
            if (w.run && !w.bad && lane == 0) pscr[w.nent - 1] = (IMSAME_MOVE_DIAG << 30) | (uint32_t)w.run;
            wv_mem_sync();
            if (!valid[h]) continue;
            bool acc = false;
            if (!w.bad)
                acc = (uint32_t)yl[h] < P.n_minlen && (uint32_t)w.len >= P.minlen[yl[h]] &&
                      (uint32_t)w.len < P.n_minident && (uint32_t)w.idn >= P.minident[w.len];
            if (w.bad && lane == 0) wv_atomic_or(P.flags, 2u);
            uint32_t poff = 0, plen = 0;
            if (acc && P.want_paths) {
                uint32_t o = 0;
                if (lane == 0) {
                    o = wv_atomic_add(P.paths_used, (uint32_t)w.nent);
                    if (o + (uint32_t)w.nent > P.paths_cap) { wv_atomic_or(P.flags, 1u); o = 0xFFFFFFFFu; }
                }
                o = wv_first(o);
                if (o != 0xFFFFFFFFu) {
                    for (int k = lane; k < w.nent; k += 64) P.paths[o + k] = pscr[k];
                    poff = o; plen = (uint32_t)w.nent;
                } else {                              // arena full: the host re-walks this pair
                    poff = 0xFFFFFFFFu; plen = (uint32_t)w.nent;
                }
            }
            if (lane == 0) {
                const int M = 2 * max(xl[h], yl[h]);
                const int tail = w.px + w.py;         // one of them is 0
                imsame_read_result r;
                r.db_seq = sid[h]; r.score = bscore[h]; r.bx = (uint32_t)bx[h]; r.by = (uint32_t)by[h];
                r.length = (uint32_t)w.len; r.identities = (uint32_t)w.idn;
                r.igaps = (uint32_t)w.ig; r.egaps = (uint32_t)w.eg;
                r.head_x = (uint32_t)(M - ((xl[h] - 1 - bx[h]) + w.len + tail));
                r.head_y = (uint32_t)(M - ((yl[h] - 1 - by[h]) + w.len + tail));
                r.ylen = (uint32_t)yl[h]; r.status = acc ? 1u : 2u;
                r.path_off = poff; r.path_len = plen;
                P.out[cidx[h]] = r;
            }
        }
        wv_mem_sync();
    }
}

#ifndef IMSAME_WAVE_EMU
#ifndef NWP_WAVES_PER_EU
#define NWP_WAVES_PER_EU 3
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NWP_WAVES_PER_EU)))
void nwp_kernel(NwLaunch P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    const uint32_t slot = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + wib);   // wave-uniform
    nwp_wave(P, smem + wib * nwl_wave_lds(P.xstride), lane, slot);
}
#endif
