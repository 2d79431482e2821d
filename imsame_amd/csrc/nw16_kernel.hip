// nw16_kernel.hip -- IMSAME's NW + backtracking for short reads (one strip,
// ylen <= NW_W/2) on PACKED PAIRS: every 32-bit register holds the same cell
// of two candidates, A in bits 0-15 and B in bits 16-31, and the recurrence
// runs on v_pk_*_i16 / bitwise forms.  Included by imsame_dev.hip (and by
// tests/emu/wave_emu.cpp under IMSAME_WAVE_EMU) after nw_kernel.hip.
//
// Reference: NW              alignmentFunctions.c:389-489
//            backtrackingNW  alignmentFunctions.c:493-560
//
// Why: on gfx950 v_max_i32, v_cndmask, v_cmp and every v_pk_*_i16 form cost
// the same ~4.2 cycles per wave instruction (scripts/micro/valu_rate.hip),
// so a packed op does two cells for the price of one.  The int32 sweep of
// nw_kernel.hip spends ~30 VALU per cell; this one 25 per PAIR of cells.
//
// Mapping: as nw_kernel.hip (a group of G lanes, NW_K columns per lane, one
// step = one row per lane with a one-lane skew, mf crossing lanes by DPP
// wave_shr:1), but each group carries candidates c = 2g and 2g+1 of its wave's
// share.  The two halves share the row index i and column index j, so every
// row/column constant (gap terms, sentinels) is the same in both halves; only
// the bases differ.  Records are staged in LDS as interleaved 2-bit codes
// (u16 per row: A in byte 0, B in byte 1).
//
// Per cell (both halves at once): s(X_i, Y_j) = v_perm of a constant table by
// (x ^ y) codes; l0/u0 adds; lu = max(l0,u0); T = max(d0,lu) + s; every
// decision is the sign of a packed difference turned into a 0xFFFF mask
// (v_pk_ashrrev 15) that selects by v_bfi and drops a traceback bit by
// v_and_or.  Traceback nibble (per half, cells 0-3 in dword 0, cell 4 in
// dword 1 of the lane's two-dword slot):
//     bit 0  NOT diagonal (d0 < max(l0, u0))
//     bit 1  up beats left (u0 > l0)   -- the move when bit 0 is set
//     bit 2  U: mc[j-1] took row i-2 here (as nw_kernel.hip)
//     bit 3  NOT L: mf kept its value after this cell (L = !bit 3)
// nib16_canon() turns it into nw_kernel.hip's nibble for the shared walk.
//
// Range: scores are int16.  The host picks this kernel only when every value
// of the launch (including the garbage rows/columns a lockstep group computes
// past a shorter candidate, which are DP values of an extended problem) stays
// within +-R, R <= 8191, so values, sentinels (NW16_BIG = 2^14) and every
// compared difference fit (nw16_fits); otherwise nw_kernel.hip runs.

#define NW16_BIG 16384

// does the launch fit the int16 path?  (all gap terms non-positive)
__host__ static inline bool nw16_fits(int64_t ig, int64_t eg, uint64_t xcap, uint64_t ymax) {
    if (ig > 0 || eg > 0 || ymax > (uint64_t)NW_W / 2 || ymax == 0) return false;
    const uint64_t G = (ymax + NW_K - 1) / NW_K, ycols = G * NW_K;
    const uint64_t aig = (uint64_t)(-ig), aeg = (uint64_t)(-eg);
    if (aig > 8191 || aeg > 8191) return false;
    const uint64_t R = 4 * ycols + aig + aeg * (xcap + 64 + ycols) + 16;
    return R <= 8191;
}

WV_DEVICE uint32_t pk1(int v) { return (uint32_t)(uint16_t)v * 0x10001u; }
WV_DEVICE uint32_t pk2(int lo, int hi) { return (uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16); }
WV_DEVICE int pk_half(uint32_t v, int h) { return (int)(int16_t)(h ? (v >> 16) : (v & 0xFFFFu)); }
WV_DEVICE uint32_t base_code(uint8_t b) { return (b >> 1) & 3u; }          // A0 C1 T2 G3: distinct

// score table for v_perm: selector byte d = xcode ^ ycode picks the low byte
// (d in 0..3) and, with bit 2 set, the high byte (4..7) of s = d ? -4 : +4
#define NW16_TBL_LO 0xFCFCFC04u
#define NW16_TBL_HI 0xFFFFFF00u

// nibble (this file's layout) -> nw_kernel.hip's nibble
WV_DEVICE uint32_t nib16_canon(uint32_t n) {
    const uint32_t mv = (n & 1u) ? ((n & 2u) ? 1u : 2u) : 0u;
    return mv | (n & 4u) | ((n & 8u) ? 0u : 8u);
}

// traceback of half h of group g: slot = steps x 64 lanes x 2 dwords
struct TbAcc16 {
    const uint32_t *tb; const uint16_t *X; const uint8_t *Y; int g, G, h;
    __device__ uint32_t nib(int i, int j) const {
        const int l = j / NW_K, s = j - l * NW_K;
        const uint32_t w = tb[((uint32_t)(i + l) * 64u + (uint32_t)(g * G + l)) * 2u + (s >> 2)];
        return nib16_canon((w >> (16 * h + 4 * (s & 3))) & 0xFu);
    }
    __device__ bool match(int i, int j) const { return ((X[i] >> (8 * h)) & 3u) == base_code(Y[j]); }
};

__host__ __device__ static inline size_t nw16_wave_lds(int GPW, int xstride) {
    return (size_t)GPW * 2 * xstride + 64 * 8 * 4;
}

// LAST4: every read length of the launch is a multiple of NW_K, so each
// candidate's last column is slot NW_K-1 of its owner lane (no select).
template <bool LAST4>
__device__ void nw16_wave(const NwLaunch &P, uint8_t *wsm, const int lane, const uint32_t slot) {
    const int G = P.G, GPW = P.GPW;
    const int g = lane / G, gl = lane - g * G;
    const bool in_group = g < GPW;
    const int gg = in_group ? g : 0;
    int *red = (int *)(wsm + (size_t)GPW * 2 * P.xstride);          // 64 lanes x 8 ints
    uint32_t *tbw = P.tb + (uint64_t)slot * P.tb_wave_dw;
    const int ig = P.igap, eg = P.egap;

    for (;;) {
        uint32_t base = 0;
        if (lane == 0) base = wv_atomic_add(P.counter, (uint32_t)(2 * GPW));
        base = wv_first(base);
        if (base >= P.n_cand) break;
        // candidates of the two halves; an absent B repeats A (never written)
        bool valid[2];
        uint32_t cidx[2], sid[2] = {0, 0};
        int xl[2] = {0, 0}, yl[2] = {0, 0};
        const uint8_t *Yp[2] = {P.q, P.q}, *Xg[2] = {P.db, P.db};
        for (int h = 0; h < 2; ++h) {
            cidx[h] = base + 2 * g + h;
            valid[h] = in_group && cidx[h] < P.n_cand;
            const uint32_t c = valid[h] ? cidx[h] : cidx[0];
            if (valid[0]) {
                const uint32_t rd = P.cand_read[c];
                sid[h] = P.cand_sid[c];
                const uint64_t xo = P.db_start[sid[h]];
                xl[h] = (int)(P.db_start[sid[h] + 1] - xo);
                Xg[h] = P.db + xo;
                const uint64_t yo = P.q_start[rd];
                Yp[h] = P.q + yo; yl[h] = (int)(P.q_start[rd + 1] - yo);
            }
        }
        const int xlp = max(xl[0], xl[1]);
        // an idle group (no candidate) reads group 0's record, so its lockstep
        // garbage stays a bounded DP like everyone else's
        uint16_t *X16 = (uint16_t *)wsm + (size_t)(valid[0] ? g : 0) * P.xstride;
        if (valid[0])
            for (int k = gl; k < xlp; k += G)
                X16[k] = (uint16_t)(base_code(Xg[0][min(k, xl[0] - 1)]) | (base_code(Xg[1][min(k, xl[1] - 1)]) << 8));
        wv_lds_sync();

        int xmax = valid[0] ? xlp : 0, xmin = valid[0] ? min(xl[0], xl[1]) : INT_MAX;
        for (int o = 32; o > 0; o >>= 1) {
            xmax = max(xmax, wv_shfl_xor(xmax, o));
            xmin = min(xmin, wv_shfl_xor(xmin, o));
        }

        // ------------------------------------------------------------ sweep
        const int j0 = gl * NW_K;
        const bool leadc0 = gl == 0;
        const int xcl = max(xlp - 1, 0);
        uint32_t yreg[NW_K], cJ[NW_K], colc[NW_K], lastm[NW_K];
        bool ownC[2], lact[2];
        for (int h = 0; h < 2; ++h) {
            ownC[h] = valid[0] && yl[h] >= 2 && yl[h] - 1 >= j0 && yl[h] - 1 < j0 + NW_K;
            lact[h] = valid[0] && j0 < yl[h];
        }
#pragma unroll
        for (int s = 0; s < NW_K; ++s) {
            const int j = j0 + s;
            const uint32_t ya = (valid[0] && j < yl[0]) ? base_code(Yp[0][j]) : 0u;
            const uint32_t yb = (valid[0] && j < yl[1]) ? base_code(Yp[1][j]) : 0u;
            yreg[s] = ya | ((ya | 4u) << 8) | (yb << 16) | ((yb | 4u) << 24);
            cJ[s] = pk1((j <= 1) ? -NW16_BIG : ig + (j - 1) * eg);      // left needs j > 1 (:443)
            colc[s] = pk1(-eg * (j - 1));
            lastm[s] = ((ownC[0] && yl[0] - 1 - j0 == s) ? 0x0000FFFFu : 0u) |
                       ((ownC[1] && yl[1] - 1 - j0 == s) ? 0xFFFF0000u : 0u);
        }
        // row 0 (:404-413)
        uint32_t xrow = valid[0] ? X16[0] : 0u;
        const uint32_t xsel0 = wv_perm(xrow, xrow, 0x01010000u);
        uint32_t yprev = 0;
        if (valid[0] && j0 > 0) {
            const uint32_t ya = base_code(Yp[0][min(j0 - 1, yl[0] - 1)]), yb = base_code(Yp[1][min(j0 - 1, yl[1] - 1)]);
            yprev = ya | ((ya | 4u) << 8) | (yb << 16) | ((yb | 4u) << 24);
        }
        const uint32_t t0prev = wv_perm(NW16_TBL_HI, NW16_TBL_LO, xsel0 ^ yprev);
        uint32_t A[NW_K], B[NW_K], C[NW_K], mcS[NW_K], mcAdj[NW_K];
#pragma unroll
        for (int s = 0; s < NW_K; ++s) {
            A[s] = wv_perm(NW16_TBL_HI, NW16_TBL_LO, xsel0 ^ yreg[s]);
            B[s] = A[s]; C[s] = A[s];
        }
#pragma unroll
        for (int s = 0; s < NW_K; ++s) {
            mcS[s] = (s == 0) ? t0prev : A[s - 1];
            mcAdj[s] = mcS[s];
            if (j0 + s == 1) mcS[s] = pk1(NW16_BIG);             // mc[0] is never updated (:476)
        }
        uint32_t I1 = t0prev, I2 = t0prev, I3 = t0prev;
        uint32_t outT = A[NW_K - 1], outMS = 0, outMA = 0;
        const int tend = xmax - 1 + G;
        xrow = valid[0] ? X16[min(max(1 - gl, 0), xcl)] : 0u;
        uint32_t bestC = pk1(-NW16_BIG), bestCi = 0, ipk = pk1(1 - gl);
        int bestR[2] = {INT_MIN, INT_MIN}, bestRj[2] = {0, 0};
        const uint32_t limp = pk2(xl[0] - 2, xl[1] - 2);
        uint32_t cIrun = 0, rcrun = 0;
        const uint32_t egp = pk1(eg);
        uint2 *tb2 = (uint2 *)tbw;

        auto step = [&](const bool PRE, const bool CAREFUL, const int t, uint32_t (&cur)[NW_K],
                        const uint32_t (&own)[NW_K], const uint32_t (&own2)[NW_K], uint32_t &in0, const uint32_t in1,
                        const uint32_t in2) {
            const uint32_t sN = (uint32_t)wv_shr1((int)outT), mS = (uint32_t)wv_shr1((int)outMS),
                           mA = (uint32_t)wv_shr1((int)outMA);
            const int i = t - gl;
            const uint32_t xsel = wv_perm(xrow, xrow, 0x01010000u);
            xrow = CAREFUL ? X16[min(max(i + 1, 0), xcl)] : X16[i + 1];       // next row, read ahead
            const bool pre = PRE && i < 1;
            uint32_t cIp, rowc2p;
            if (CAREFUL) {
                cIp = pk1((i <= 1) ? -NW16_BIG : ig + (i - 1) * eg);          // up needs i > 1 (:449)
                rowc2p = pk1(-eg * (i - 2));
                cIrun = pk1(ig + i * eg); rcrun = pk1(-eg * (i - 1));
            } else {
                cIp = cIrun; rowc2p = rcrun;
                cIrun = pk_add(cIrun, egp); rcrun = pk_sub(rcrun, egp);
            }
            uint32_t mfS = mS, mfAdj = mA, w0 = 0, w1 = 0;
#pragma unroll
            for (int s = 0; s < NW_K; ++s) {
                const uint32_t d0 = (s == 0) ? in1 : own[s - 1];     // T[i-1][j-1]
                const uint32_t u2 = (s == 0) ? in2 : own2[s - 1];    // T[i-2][j-1]
                const uint32_t tl = (s == 0) ? sN : cur[s - 1];      // T[i][j-1]
                const uint32_t sc = wv_perm(NW16_TBL_HI, NW16_TBL_LO, xsel ^ yreg[s]);
                const uint32_t l0 = pk_add(mfAdj, cJ[s]);              // left - s (:444)
                const uint32_t u0 = pk_add(mcAdj[s], cIp);             // up   - s (:450)
                const uint32_t lu = pk_max(l0, u0);
                uint32_t v = pk_add(pk_max(d0, lu), sc);
                if (s == 0) v = leadc0 ? sc : v;                      // column 0 (:426)
                cur[s] = pre ? own[s] : v;
                const uint32_t ndm = pk_neg_mask(pk_sub(d0, lu));      // not diagonal (:457-472)
                const uint32_t upm = pk_neg_mask(pk_sub(l0, u0));      // up > left
                // column max of column j-1 over rows <= i-2, strict > (:476-480)
                const uint32_t cum = pk_neg_mask(pk_sub(mcS[s], u2));
                mcAdj[s] = wv_bfi(cum, pk_add(u2, rowc2p), mcAdj[s]);
                mcS[s] = pk_max(mcS[s], u2);
                // row state for column j+1: tested on row i, taken from row i-1 (:434-438)
                const uint32_t nclm = pk_neg_mask(pk_sub(tl, mfS));
                mfAdj = wv_bfi(nclm, mfAdj, pk_add(d0, colc[s]));
                mfS = wv_bfi(nclm, mfS, d0);
                if (s == 0) mfS = leadc0 ? pk1(-NW16_BIG) : mfS;    // then mf = T[i-1][0]
                const uint32_t sh = 4u * (uint32_t)(s & 3);
                uint32_t &w = (s < 4) ? w0 : w1;
                w = wv_and_or(ndm, 0x10001u << sh, w);
                w = wv_and_or(upm, 0x20002u << sh, w);
                w = wv_and_or(cum, 0x40004u << sh, w);
                w = wv_and_or(nclm, 0x80008u << sh, w);
            }
            // rows outside [1, xlen) are never read; 32-bit byte offset from the
            // wave-uniform slot base (global_store saddr form)
            *(uint2 *)((uint8_t *)tb2 + ((uint32_t)t * 512u + (uint32_t)lane * 8u)) = make_uint2(w0, w1);
            // last column (rows 1 .. xlen-2) and last row (:481-484)
            uint32_t vl = cur[LAST4 ? NW_K - 1 : 0];
            if (!LAST4)
#pragma unroll
                for (int s = 1; s < NW_K; ++s) vl = wv_bfi(lastm[s], cur[s], vl);
            uint32_t km = pk_neg_mask(pk_sub(vl, bestC));             // keep where vl < best (">=" takes)
            if (CAREFUL) {
                km |= pk_neg_mask(pk_sub(limp, ipk)) | pk_neg_mask(pk_sub(ipk, pk1(1)));
                if (i >= 1 && (i == xl[0] - 1 || i == xl[1] - 1)) {
                    for (int h = 0; h < 2; ++h) {
                        if (!lact[h] || i != xl[h] - 1) continue;
#pragma unroll
                        for (int s = 0; s < NW_K; ++s) {
                            const int j = j0 + s, val = pk_half(cur[s], h);
                            if (j >= 1 && j < yl[h] && val >= bestR[h]) { bestR[h] = val; bestRj[h] = j; }
                        }
                    }
                }
            }
            bestC = wv_bfi(km, bestC, vl);
            bestCi = wv_bfi(km, bestCi, ipk);
            ipk = pk_add(ipk, 0x10001u);
            in0 = pre ? in1 : sN;
            outT = cur[NW_K - 1]; outMS = mfS; outMA = mfAdj;
        };
        // (cur, own, own2) and (in0, in1, in2) rotate every step; every loop
        // advances t by 3 so the rotation phase carries over
        int t = 1;
        for (; t + 2 < tend && t <= G; t += 3) {                 // skewed start: lanes may be before row 1
            step(true, true, t, A, B, C, I3, I1, I2);
            step(true, true, t + 1, C, A, B, I2, I3, I1);
            step(true, true, t + 2, B, C, A, I1, I2, I3);
        }
        for (; t + 2 <= xmin - 2; t += 3) {                      // every lane inside every record
            step(false, false, t, A, B, C, I3, I1, I2);
            step(false, false, t + 1, C, A, B, I2, I3, I1);
            step(false, false, t + 2, B, C, A, I1, I2, I3);
        }
        for (; t + 2 < tend; t += 3) {
            step(false, true, t, A, B, C, I3, I1, I2);
            step(false, true, t + 1, C, A, B, I2, I3, I1);
            step(false, true, t + 2, B, C, A, I1, I2, I3);
        }
        if (t < tend) step(true, true, t, A, B, C, I3, I1, I2);
        if (t + 1 < tend) step(true, true, t + 1, C, A, B, I2, I3, I1);
        wv_mem_sync();                            // traceback written by all lanes, read by the walkers

        // best cell per half: row-major order, ">=" -> last visited wins
        for (int h = 0; h < 2; ++h) {
            red[lane * 8 + 4 * h + 0] = bestR[h];
            red[lane * 8 + 4 * h + 1] = bestRj[h];
            red[lane * 8 + 4 * h + 2] = ownC[h] ? pk_half(bestC, h) : INT_MIN;
            red[lane * 8 + 4 * h + 3] = pk_half(bestCi, h);
        }
        wv_lds_sync();
        int bscore[2], bx[2], by[2];
        for (int h = 0; h < 2; ++h) {
            int bR = INT_MIN, bRj = 0, bC = INT_MIN, bCi = 0;
            if (in_group)
                for (int k = 0; k < G; ++k) {
                    const int *e = red + (g * G + k) * 8 + 4 * h;
                    if (e[0] > bR || (e[0] == bR && e[1] > bRj)) { bR = e[0]; bRj = e[1]; }
                    if (e[2] > bC || (e[2] == bC && e[3] > bCi)) { bC = e[2]; bCi = e[3]; }
                }
            if (bR >= bC) { bscore[h] = bR; bx[h] = xl[h] - 1; by[h] = bRj; }
            else          { bscore[h] = bC; bx[h] = bCi; by[h] = yl[h] - 1; }
        }
        wv_lds_sync();
        for (int h = 0; h < 2; ++h) {
            const TbAcc16 acc16 = {tbw, X16, Yp[h], gg, G, h};
            nw_finish(P, acc16, xl[h], yl[h], valid[h], gg, gl, G, bscore[h], bx[h], by[h], cidx[h], sid[h]);
        }
        wv_lds_sync();
    }
}

// Launch shape: G lanes per group, GPW groups (2*GPW candidates) per wave
__host__ static inline NwShape nw16_shape(uint32_t ymax, uint32_t xcap) {
    NwShape s;
    s.G = (int)((ymax + NW_K - 1) / NW_K);
    if (s.G < 1) s.G = 1;
    s.GPW = 64 / s.G; s.nstr = 1;
    s.xcap = xcap < 2 ? 2 : (int)xcap;
    s.xstride = (s.xcap + 15) & ~15;
    while (s.GPW > 1 && (size_t)s.GPW * 2 * s.xstride > 16384) s.GPW--;
    s.steps = s.xcap + s.G;
    return s;
}
// traceback dwords per wave slot (two per lane per step)
__host__ static inline uint64_t nw16_tb_words(const NwShape &s) { return (uint64_t)s.steps * 64 * 2; }

#ifndef IMSAME_WAVE_EMU
#ifndef NW16_WAVES_PER_EU
#define NW16_WAVES_PER_EU 4
#endif
template <bool LAST4>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NW16_WAVES_PER_EU)))
void nw16_kernel(NwLaunch P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    const uint32_t slot = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + wib);   // wave-uniform
    nw16_wave<LAST4>(P, smem + wib * nw16_wave_lds(P.GPW, P.xstride), lane, slot);
}
#endif
