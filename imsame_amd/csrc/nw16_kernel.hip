// nw16_kernel.hip -- IMSAME's NW + backtracking for short reads (one strip,
// ylen <= NW_W/2) on PACKED PAIRS: every 32-bit register holds the same cell
// of two candidates, A in bits 0-15 and B in bits 16-31, and the recurrence
// runs on v_pk_*_i16 / bitwise forms.  Included by imsame_dev.hip (and by
// tests/emu/wave_emu.cpp under IMSAME_WAVE_EMU) after nw_kernel.hip.
//
// Reference: NW              alignmentFunctions.c:389-489
//            backtrackingNW  alignmentFunctions.c:493-560
//
// Why: on gfx950 the NW sweep is bound by VALU issue, and v_max_i32,
// v_cndmask, v_cmp and every v_pk_*_i16 form issue at the same ~4.2 cycles
// per wave instruction (scripts/micro/valu_rate.hip; in mixed streams even
// the "full-rate" adds cost ~3.5-4), so a packed op does two cells for the
// price of one and the instruction count is the cost model.
//
// Mapping: a group of G lanes carries candidates 2g and 2g+1 of its wave's
// share; lane gl owns K = 10 consecutive columns (K = 5 for latency-bound
// launches: twice the waves, each half as long -- nw16_k) and walks the rows with
// a one-lane skew (step t: row i = t - gl); the row state crosses lanes by
// DPP wave_shr:1.  The two halves share the row and column indices, so every
// row/column constant is common; only the bases differ.  Records are staged
// in LDS as one byte per row per pair (2-bit codes, A in bits 0-1, B in 2-3).
//
// State per cell (both halves at once), with the reference's gap terms kept
// as DRIFTING values so no per-column or per-row constant is needed:
//     l0 = left - s = mf.score + ig + (j - mf.y - 1)*eg    (flows along the row)
//          next column: taken ? d0 + ig + eg : l0 + eg        (:434-438, :444)
//     u0 = up - s   = mc.score + ig + (i - mc.x - 1)*eg    (one per column)
//          next row:    U     ? u2 + ig + 2eg : u0 + eg       (:450, :476-480)
// T = max(d0, max(l0, u0)) + s, s = v_perm of a constant table by (x ^ y)
// codes; each decision is the sign of a packed difference, turned into a
// 0xFFFF mask (v_pk_ashrrev 15) where a select (v_bitop3) needs it.
//
// Traceback, three dwords per lane per step (0.6 B/cell; K = 5: WM and WU only):
//   WM  cells 0-7: bit s = NOT-diag(A), 8+s NOT-diag(B), 16+s up(A), 24+s up(B)
//       -- one v_perm turns the four signs of (d0 - lu, l0 - u0) into 0xFF/0x00
//          bytes (selectors 8-11 replicate bits 15/31/47/63)
//   WU  cells 0-7: bit s = U(A), 8+s NOT-L(A), 16+s U(B), 24+s NOT-L(B)
//   WX  cells 8-9 (s' = s - 8): moves at s', 8+s', 16+s', 24+s';
//       U(A) 2+s', NOT-L(A) 4+s', U(B) 18+s', NOT-L(B) 20+s'
// with U = mc[j-1] took (T[i-2][j-1], row i-2) at this cell and L = mf took
// (T[i-1][j-1], col j-1) after it, as nw_kernel.hip; TbAcc16 hands the walk
// that kernel's nibble.
//
// Two passes (TWO, the default): the full sweep writes no traceback -- it
// keeps the DP values, the best cell and, every nw16_ck(K) steps, a checkpoint of
// the wave's register state (4K+5 dwords per lane) -- and a second sweep
// restarts each half from the last checkpoint at least band_w rows above its
// best cell, per half (its own rows: two LDS row reads and per-half row masks),
// and writes the traceback of those ~band_w + nw16_ck(K) + G steps only.  The
// walk reads only rows the second sweep wrote (TbAcc16::has); a path that
// leaves them is LOST and the wave redoes the second sweep over 4 bands, then
// from row 1 (same values: the state restored is the state the first sweep
// had).  The
// move bits and their packing are 6 of the 23 instructions per cell pair, so
// the first sweep issues ~190 VALU per step instead of 250, and ~90 % of the
// steps are first-sweep steps at C2 (2000-row records, 150-column reads).
//
// Predicted window (P.cand_row): the seed hit that made a candidate puts the
// read's first base on record row cand_row, so an accepted read's path runs
// over rows ~[cand_row, cand_row + ylen) and its best cell sits at the bottom
// of them.  The host orders the queue by that row (P.perm), so a wave's eight
// candidates predict nearly the same rows, and the FIRST sweep writes the
// traceback of the union of their windows (~230 of ~2000 steps, at the
// one-pass cost per step).  A half whose best cell lies inside the window
// walks it directly (TbAcc16 bounds [t0, t1)); a half whose best cell is
// elsewhere or whose walk leaves the window falls back to the second sweep
// above.  Same DP values either way, so the same bits.
//
// Range: scores are int16.  The host picks this kernel only when every value
// of the launch (including the garbage rows/columns a lockstep group computes
// past a shorter candidate, which are DP values of an extended problem) stays
// within +-R, R <= 8191, so values, sentinels (NW16_BIG = 2^14) and every
// compared difference fit (nw16_fits); otherwise nw_kernel.hip runs.

#define NW16_K   10               // columns per lane (the full-chip launches)
#define NW16_K5  5                // columns per lane of the latency-bound launches (nw16_k)
// The latency form (round 6): 3 columns per lane, one candidate pair per
// wave (G = 50 at 150 bp).  A lone wave issues its row step serially -- ~16
// VALU per column plus ~20 per step -- so a launch of a few hundred waves
// lasts about xlen steps of that chain: 5 columns cost ~100 VALU per step, 3
// cost ~70.  For the small launches of the last rounds (imsame_dev.hip:nw16_k).
#define NW16_K3  3
#define NW16_K3_YMAX 150          // G <= 50: nw16_ck(3) + G <= 64 (the range proof's extra rows)
#define NW16_BIG 16384
// Checkpoint interval of the first sweep, per column form (steps; even: the
// rotation period).  nw16_fits bounds the rows a second sweep runs past the
// first by CK + G <= 64: K = 5 has G <= 32 (CK 32), K = 10 G <= 16 and K = 19
// G = 8 (CK 48).  The checkpoint is 4K+5 dwords (dI is recomputed on restore):
// round 3 wrote 5K+5 every 24 steps (0.46 B/cell at C2), 4K+5 every 48 is
// ~0.19 B/cell, for ~8 more second-sweep rows per half on average -- only
// for the halves the first sweep's predicted window does not cover.
// (K = 3: G <= 50, so CK 14)
__host__ __device__ constexpr int nw16_ck(int K) { return K <= 3 ? 14 : K <= 5 ? 32 : 48; }
// dwords of wave state per lane in a checkpoint (A, B, mcS, u0 per column; I1,
// I2, outT, outMS, outL); dI is a function of A and I2 there (save())
__host__ __device__ constexpr int nw16_nst(int K) { return 4 * K + 5; }
// K <= 10: WM, WU (+ WX for cells 8-9); K > 10 (the 19-column form): WM_b, WU_b
// for each block b of 8 cells (cells 8b .. 8b+7 at bits q = s - 8b)
__host__ __device__ constexpr int nw16_nrec(int K) { return K <= 8 ? 2 : K <= 10 ? 3 : 2 * ((K + 7) / 8); }
// The 19-column form (nw16_k19): 8 lanes per candidate pair, 8 groups per
// wave -- all 64 lanes busy at 150 bp, where K = 10 leaves 4 of 64 idle -- and
// the per-step work (DPP, row code, best cell) spread over 19 columns instead
// of 10.  Lane gl owns columns [gl*K - OFF, gl*K - OFF + K): the OFF leading
// columns of lane 0 are padding (never read), so a read of length G*K - OFF
// ends in slot K-1 of its last lane (the LAST form) -- 150 = 8*19 - 2.
#define NW16_K19 19
#define NW16_K19_OFF 2
#define NW16_K19_YLEN (8 * NW16_K19 - NW16_K19_OFF)
#define NW16_NOROW INT32_MIN      // cand_row: no prediction
#define NW16_WIN_UP 32            // window rows above the predicted first row
#define NW16_WIN_DOWN 24          // ... and below the predicted last row
#define NW16_WIN_MAX 448          // longest window (steps) a wave writes in its first sweep
#define NW16_WIN_BOTTOM 40        // rows above the last one for an unpredicted candidate
#define NW16_BAND2 4              // the second sweep's retry band, in bands

// does the launch fit the int16 path?  (all gap terms non-positive)
__host__ static inline bool nw16_fits(int64_t ig, int64_t eg, uint64_t xcap, uint64_t ymax, int K = NW16_K) {
    if (ig > 0 || eg > 0 || ymax > (uint64_t)NW_W / 2 || ymax == 0) return false;
    const uint64_t G = (ymax + K - 1) / K, ycols = G * K;
    const uint64_t aig = (uint64_t)(-ig), aeg = (uint64_t)(-eg);
    if (aig > 8191 || aeg > 8191) return false;
    // |T| <= 4*ycols; l0 >= -T - |ig| - |eg|*ycols; u0 drifts at most over
    // xcap + 64 rows (lockstep garbage rows included -- a second sweep runs at
    // most nw16_ck(K) + G <= 64 rows past the first one)
    // and takes u2 + ig + 2eg.  ycols at K = 10 bounds ycols at K = 5 (K = 19
    // asks with its own ycols; its padding columns never feed a real one).
    const uint64_t R = 4 * ycols + aig + aeg * (xcap + 64 + ycols + 2) + 16;
    return R <= 8191;
}

WV_DEVICE uint32_t pk1(int v) { return (uint32_t)(uint16_t)v * 0x10001u; }
WV_DEVICE uint32_t pk2(int lo, int hi) { return (uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16); }
WV_DEVICE int pk_half(uint32_t v, int h) { return (int)(int16_t)(h ? (v >> 16) : (v & 0xFFFFu)); }
// DP values are held BIASED by 2^15 (each half's top bit flipped, an xor):
// every value of a launch lies in [-NW16_BIG - R, NW16_BIG] (nw16_fits: R <=
// 8191, sentinels and drift included), so a biased half stays in [8193,
// 49152].  Unsigned maxes order them, differences (and their signs) are the
// unbiased ones, and adding a gap constant is a plain 32-bit subtract of its
// magnitude -- no borrow can cross from one half into the other -- which
// issues in half the cycles of v_pk_add_i16 (§4.1, profiles/r06_valu_rate.txt).
#define NW16_H 0x80008000u
WV_DEVICE int pk_score(uint32_t v, int h) { return (int)(h ? (v >> 16) : (v & 0xFFFFu)) - 32768; }
WV_DEVICE uint32_t base_code(uint8_t b) { return (b >> 1) & 3u; }          // A0 C1 T2 G3: distinct

// The substitution score of a cell pair.  NW16_ROWTAB (the default, round
// 6): each step builds two ROW tables from the row's record codes -- tlo =
// 8 << 8*xA (byte xA of A's table is 8, the others 0) and thi = 8 << 8*xB --
// and each column keeps a constant selector ysel = [yA, 0x0C, 4 + yB, 0x0C],
// so one v_perm gives [8*(xA==yA), 0, 8*(xB==yB), 0] and one v_add3_u32 adds
// it with the -4 of a mismatch folded in (max + s8 - 0x00040004; biased
// halves never carry across).  Per cell pair: perm + add3 instead of xor +
// perm + pk_add -- one instruction fewer, for 4 per step to build the tables
// (3 before: the xor selector).  The LDS record byte of a row pair is xA << 3
// | xB << 5, so tlo is one v_lshlrev (the shift uses the low 5 bits).
// Otherwise (NW16_ROWTAB=0): a constant table indexed by xcode ^ ycode.
#ifndef NW16_ROWTAB
#define NW16_ROWTAB 1
#endif
#define NW16_TBL_LO 0xFCFCFC04u
#define NW16_TBL_HI 0xFFFFFF00u
#if NW16_ROWTAB
#define NW16_XSH_A 3              // bit of A's record code in the LDS row byte
#define NW16_XSH_B 5              // ... and of B's
#else
#define NW16_XSH_A 0
#define NW16_XSH_B 2
#endif
#define NW16_XM_A (3u << NW16_XSH_A)
#define NW16_XM_B (3u << NW16_XSH_B)
// a row pair's table (ROWTAB: tlo, thi; else the xor selector in lo)
struct Nw16Row { uint32_t lo, hi; };
WV_DEVICE Nw16Row nw16_row(uint32_t xb) {
#if NW16_ROWTAB
    return {8u << (xb & 31u), 8u << ((xb >> 2) & 0x18u)};
#else
    return {wv_perm(xb >> 2, xb & 3u, 0x04040000u), 0u};
#endif
}
// a column's constant operand for the codes ya, yb of its two halves
WV_DEVICE uint32_t nw16_ycol(uint32_t ya, uint32_t yb) {
#if NW16_ROWTAB
    return ya | (0x0Cu << 8) | ((yb + 4u) << 16) | (0x0Cu << 24);
#else
    return ya | ((ya | 4u) << 8) | (yb << 16) | ((yb | 4u) << 24);
#endif
}
// the cell pair's score term (ROWTAB: 0 / 8 per half; else +-4 as int16)
WV_DEVICE uint32_t nw16_sc(const Nw16Row &r, uint32_t ycol) {
#if NW16_ROWTAB
    return wv_perm(r.hi, r.lo, ycol);
#else
    return wv_perm(NW16_TBL_HI, NW16_TBL_LO, r.lo ^ ycol);
#endif
}
// T = max + score (biased halves)
WV_DEVICE uint32_t nw16_add_sc(uint32_t m, uint32_t sc) {
#if NW16_ROWTAB
    return m + sc + 0xFFFBFFFCu;                  // + s8 - 0x00040004: one v_add3_u32
#else
    return pk_add(m, sc);
#endif
}
// the biased score itself (row 0, column 0: T = score)
WV_DEVICE uint32_t nw16_sc_biased(uint32_t sc) {
#if NW16_ROWTAB
    return sc + 0x7FFC7FFCu;                      // s8 - 4 + 2^15 per half
#else
    return sc ^ 0x80008000u;
#endif
}

// cell s of half h in one lane's traceback words of a step (layout above) ->
// nw_kernel.hip's nibble: move (0 diag, 1 up, 2 left) | U << 2 | L << 3
template <int K>
WV_DEVICE uint32_t tb16_nib(const uint32_t *w, const int s, const int h) {
    uint32_t nd, up, U, nL;
    if (K > 10) {
        const uint32_t wm = w[2 * (s >> 3)], wu = w[2 * (s >> 3) + 1], q = (uint32_t)(s & 7);
        nd = (wm >> (8 * h + q)) & 1u; up = (wm >> (16 + 8 * h + q)) & 1u;
        U = (wu >> (16 * h + q)) & 1u; nL = (wu >> (16 * h + 8 + q)) & 1u;
    } else if (s < 8) {
        const uint32_t wm = w[0], wu = w[1];
        nd = (wm >> (8 * h + s)) & 1u; up = (wm >> (16 + 8 * h + s)) & 1u;
        U = (wu >> (16 * h + s)) & 1u; nL = (wu >> (16 * h + 8 + s)) & 1u;
    } else {
        const uint32_t wx = w[2], q = (uint32_t)(s - 8);
        nd = (wx >> (8 * h + q)) & 1u; up = (wx >> (16 + 8 * h + q)) & 1u;
        U = (wx >> (16 * h + 2 + q)) & 1u; nL = (wx >> (16 * h + 4 + q)) & 1u;
    }
    return (nd ? (up ? 1u : 2u) : 0u) | (U << 2) | ((nL ^ 1u) << 3);
}

// traceback of half h of group g (layout above) -> nw_kernel.hip's nibble
// t0: step of the sweep that wrote record 0 (0: one pass, steps indexed by t;
// two passes: the half's restart step, cells before it were not written)
template <int K, int OFF = 0>
struct TbAcc16 {
    const uint32_t *tb; const uint8_t *X; const uint8_t *Y; int g, G, h, t0;
    int t1 = INT_MAX;                      // steps [t0, t1) were written
    __device__ bool has(int i, int j) const { const int t = i + (j + OFF) / K; return t >= t0 && t < t1; }
    __device__ uint32_t nib(int i, int j) const {
        const int l = (j + OFF) / K, s = (j + OFF) - l * K;
        return tb16_nib<K>(tb + ((uint32_t)(i + l - t0) * 64u + (uint32_t)(g * G + l)) * (uint32_t)nw16_nrec(K), s, h);
    }
    __device__ bool match(int i, int j) const {
        return ((X[i] >> (h ? NW16_XSH_B : NW16_XSH_A)) & 3u) == base_code(Y[j]);
    }
};

// one lane's traceback words of one step (layout above), built cell by cell
// (s is a compile-time slot after unrolling: the words stay in registers)
template <int K>
struct TbWords {
    uint32_t w[nw16_nrec(K)];
    WV_DEVICE void add(const int s, const uint32_t P2, const uint32_t mU, const uint32_t mnL) {
        if (K > 10) {
            const int b = s >> 3, q = s & 7;
            w[2 * b] = wv_and_or(P2, 0x01010101u << q, w[2 * b]);
            w[2 * b + 1] = wv_and_or(mU, 0x00010001u << q, w[2 * b + 1]);
            w[2 * b + 1] = wv_and_or(mnL, 0x01000100u << q, w[2 * b + 1]);
        } else if (s < 8) {
            w[0] = wv_and_or(P2, 0x01010101u << s, w[0]);
            w[1] = wv_and_or(mU, 0x00010001u << s, w[1]);
            w[1] = wv_and_or(mnL, 0x01000100u << s, w[1]);
        } else {
            constexpr int X = nw16_nrec(K) - 1;       // WX (K = 10; the branch is dead for K <= 8)
            const int q = s - 8;
            w[X] = wv_and_or(P2, 0x01010101u << q, w[X]);
            w[X] = wv_and_or(mU, 0x00040004u << q, w[X]);
            w[X] = wv_and_or(mnL, 0x00100010u << q, w[X]);
        }
    }
    WV_DEVICE void store(uint32_t *rec) const {
#pragma unroll
        for (int r = 0; r < nw16_nrec(K); ++r) rec[r] = w[r];
    }
};

__host__ __device__ static inline size_t nw16_wave_lds(int GPW, int xstride) {
    return (size_t)GPW * xstride + 64 * 8 * 4;
}

// LAST: every read length of the launch is a multiple of K (or, with OFF > 0,
// equals G*K - OFF), so each candidate's last column is slot K-1 of its owner
// lane (no select).  OFF: padding columns ahead of column 0 (nw16_k19).
// TWO: score-only sweep + checkpoints, then the traceback band (header).
template <int K, bool LAST, bool TWO, int OFF = 0>
__device__ __forceinline__ void nw16_wave(const NwLaunch &P, uint8_t *wsm, const int lane, const uint32_t slot) {
    constexpr int NST = nw16_nst(K), NREC = nw16_nrec(K), CK = nw16_ck(K);
    constexpr uint32_t RECB = 64u * 4u * NREC;     // traceback bytes per step
    const int G = P.G, GPW = P.GPW;
    const int g = lane / G, gl = lane - g * G;
    const bool in_group = g < GPW;
    const int gg = in_group ? g : 0;
    int *red = (int *)(wsm + (size_t)GPW * P.xstride);                // 64 lanes x 8 ints
    uint32_t *tbw = P.tb + (uint64_t)slot * P.tb_wave_dw;
    uint32_t *ckw = TWO ? P.ck + (uint64_t)slot * P.ck_wave_dw + lane : nullptr;
    const int ig = P.igap, eg = P.egap;

    // phase profile (P.prof): 0 fetch + staging + setup, 1 first sweep, 2 best-cell
    // reduction, 3 second sweep(s) incl. restore, 4 walks + results
    // (and the wave's 100 MHz real time beside its cycles: the shader clock under this load)
    unsigned long long ph[5] = {0, 0, 0, 0, 0}, tq = P.prof ? wv_clock() : 0, rt0 = P.prof ? wv_realtime() : 0;
    auto mark = [&](const int k) {
        if (P.prof) { const unsigned long long n = wv_clock(); ph[k] += n - tq; tq = n; }
    };
    for (uint32_t ntask = 0;; ++ntask) {
        if (P.slot_bits && ntask) break;          // non-persistent launch: one task per wave
        uint32_t base = 0;
        if (lane == 0) base = wv_atomic_add(P.counter, (uint32_t)(2 * GPW));
        base = wv_first(base);
        if (base >= P.n_cand) break;
        // candidates of the two halves; an absent B repeats A (never written)
        bool valid[2];
        uint32_t cidx[2], sid[2] = {0, 0};
        int xl[2] = {0, 0}, yl[2] = {0, 0}, prow[2] = {NW16_NOROW, NW16_NOROW};
        const uint8_t *Yp[2] = {P.q, P.q}, *Xg[2] = {P.db, P.db};
        for (int h = 0; h < 2; ++h) {
            cidx[h] = base + 2 * g + h;                                   // queue slot
            valid[h] = in_group && cidx[h] < P.n_cand;
        }
        for (int h = 0; h < 2; ++h) {
            const uint32_t w = valid[h] ? cidx[h] : cidx[0];
            if (valid[0]) {
                const uint32_t c = P.perm ? P.perm[w] : w;                // candidate
                cidx[h] = c;
                if (P.cand_row) prow[h] = P.cand_row[c];
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
        uint8_t *X8 = wsm + (size_t)(valid[0] ? g : 0) * P.xstride;
        if (valid[0]) {
            // 16 rows per lane and iteration: one unaligned 16-byte load per record
            // where the chunk lies inside it (else bytes clamped to its last base),
            // codes packed four per dword, one 16-byte LDS store (xstride is a
            // multiple of 16, so the chunk past xlp stays inside the group's area)
            const int nch = (xlp + 15) >> 4;
            for (int c = gl; c < nch; c += G) {
                const int k0 = c << 4;
                uint32_t w[2][4];
                for (int h = 0; h < 2; ++h) {
                    if (k0 + 16 <= xl[h]) {
                        __builtin_memcpy(w[h], Xg[h] + k0, 16);
                    } else {
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            uint32_t v = 0;
#pragma unroll
                            for (int b = 0; b < 4; ++b) v |= (uint32_t)Xg[h][min(k0 + 4 * q + b, xl[h] - 1)] << (8 * b);
                            w[h][q] = v;
                        }
                    }
                }
                uint32_t o[4];
#pragma unroll
                for (int q = 0; q < 4; ++q)   // base_code per byte: (b >> 1) & 3, A's at NW16_XSH_A, B's at _B
                    o[q] = (((w[0][q] >> 1) << NW16_XSH_A) & (NW16_XM_A * 0x01010101u)) |
                           (((w[1][q] >> 1) << NW16_XSH_B) & (NW16_XM_B * 0x01010101u));
                __builtin_memcpy(X8 + k0, o, 16);
            }
        }
        wv_lds_sync();

        int xmax = valid[0] ? xlp : 0, xmin = valid[0] ? min(xl[0], xl[1]) : INT_MAX;
        for (int o = 32; o > 0; o >>= 1) {
            xmax = max(xmax, wv_shfl_xor(xmax, o));
            xmin = min(xmin, wv_shfl_xor(xmin, o));
        }
        // wave-uniform in SGPRs: the sweep's step counter and bounds are scalar
        xmax = (int)wv_first((uint32_t)xmax); xmin = (int)wv_first((uint32_t)xmin);
        // traceback window of the first sweep: steps [tw0, tw1), both odd (the
        // loops advance t by 2 from 1); rows [lo, hi] of every candidate's
        // prediction take steps lo .. hi + G - 1
        int tw0 = INT_MAX - 2, tw1 = INT_MAX - 2;    // none: every step before "the window"
        if (TWO && P.cand_row) {
            int lo = INT_MAX, hi = INT_MIN, none = 0;
            for (int h = 0; h < 2; ++h) {
                if (!valid[h]) continue;
                if (prow[h] == NW16_NOROW) {
                    // no prediction (a weak hit: random reads' e-value passes, whose
                    // best cells mostly sit on the last row with short paths)
                    if (P.win_bottom < 0) { none = 1; continue; }
                    lo = min(lo, xl[h] - 1 - P.win_bottom);
                    hi = max(hi, xl[h] - 1);
                    continue;
                }
                lo = min(lo, prow[h] - P.win_up);
                hi = max(hi, prow[h] + yl[h] - 1 + P.win_down);
            }
            for (int o = 32; o > 0; o >>= 1) {
                lo = min(lo, wv_shfl_xor(lo, o));
                hi = max(hi, wv_shfl_xor(hi, o));
                none = max(none, wv_shfl_xor(none, o));
            }
            if (!none && lo <= hi) {
                int a = max(lo, 1), b = min(hi, xmax) + G;
                a -= (a & 1) ^ 1; b += (b & 1) ^ 1;
                if (b > a && b - a <= NW16_WIN_MAX) { tw0 = a; tw1 = b; }
            }
            tw0 = (int)wv_first((uint32_t)tw0); tw1 = (int)wv_first((uint32_t)tw1);   // wave-uniform (SGPRs)
        }
        const int tb0 = TWO ? tw0 : 0;             // step of traceback record 0

        // ------------------------------------------------------------ sweep
        const int j0 = gl * K - OFF;
        const bool leadc0 = gl == 0;
        const int xcl = max(xlp - 1, 0);
        const uint32_t NBIG = pk1(-NW16_BIG) ^ NW16_H, EGN = pk1(-eg), IGEN = pk1(-(ig + eg));   // biased; gap magnitudes
        uint32_t yreg[K], lastm[K];
        bool ownC[2], lact[2];
        for (int h = 0; h < 2; ++h) {
            ownC[h] = valid[0] && yl[h] >= 2 && yl[h] - 1 >= j0 && yl[h] - 1 < j0 + K;
            lact[h] = valid[0] && j0 < yl[h];
        }
#pragma unroll
        for (int s = 0; s < K; ++s) {
            const int j = j0 + s;
            const uint32_t ya = (valid[0] && j >= 0 && j < yl[0]) ? base_code(Yp[0][j]) : 0u;
            const uint32_t yb = (valid[0] && j >= 0 && j < yl[1]) ? base_code(Yp[1][j]) : 0u;
            yreg[s] = nw16_ycol(ya, yb);
            lastm[s] = ((ownC[0] && yl[0] - 1 - j0 == s) ? 0x0000FFFFu : 0u) |
                       ((ownC[1] && yl[1] - 1 - j0 == s) ? 0xFFFF0000u : 0u);
        }
        // row 0 (:404-413)
        uint32_t xrow = valid[0] ? X8[0] : 0u;
        const Nw16Row xr0 = nw16_row(xrow);
        uint32_t yprev = nw16_ycol(0u, 0u);
        if (valid[0] && j0 > 0) {
            const uint32_t ya = base_code(Yp[0][min(j0 - 1, yl[0] - 1)]), yb = base_code(Yp[1][min(j0 - 1, yl[1] - 1)]);
            yprev = nw16_ycol(ya, yb);
        }
        const uint32_t t0prev = nw16_sc_biased(nw16_sc(xr0, yprev));
        // The column state keeps mc's score in a frame shifted by ig + eg: dI[s]
        // = T[i-2][j-1] + ig + eg is the previous row's d0 + ig + eg of this
        // slot (the left take computes it anyway), so the column max compares
        // and takes it directly, and the up term re-based on a take is
        // dI + eg (= T[i-2][j-1] + ig + 2eg, :450) -- no row i-2 array.
        uint32_t A[K], B[K], dI[K], mcS[K], u0[K];
#pragma unroll
        for (int s = 0; s < K; ++s) {
            A[s] = nw16_sc_biased(nw16_sc(xr0, yreg[s]));
            B[s] = A[s];
        }
#pragma unroll
        for (int s = 0; s < K; ++s) {
            // mc[j-1] = (T[0][j-1], row 0); row 0 stands in for rows -1 and -2
            dI[s] = ((s == 0) ? t0prev : A[s - 1]) - IGEN;
            mcS[s] = dI[s];
            u0[s] = dI[s];                                        // its up term at row 2
            if (j0 + s == 1) mcS[s] = pk1(NW16_BIG) ^ NW16_H;            // mc[0] is never updated (:476)
        }
        uint32_t I1 = t0prev, I2 = t0prev;
        uint32_t outT = A[K - 1], outMS = 0, outL = 0;
        const int tend = xmax - 1 + G;
        xrow = valid[0] ? X8[min(max(1 - gl, 0), xcl)] : 0u;
        uint32_t bestC = pk1(-NW16_BIG) ^ NW16_H, bestCi = 0, ipk = pk1(1 - gl);
        int bestR[2] = {INT_MIN, INT_MIN}, bestRj[2] = {0, 0};
        const uint32_t limp = pk2(xl[0] - 2, xl[1] - 2);
        uint8_t *tb3 = (uint8_t *)tbw;

        auto step = [&](const bool PRE, const bool CAREFUL, const bool TB, const int t, uint32_t (&cur)[K],
                        const uint32_t (&own)[K], uint32_t &in0, const uint32_t in1) {
            const uint32_t sN = (uint32_t)wv_shr1((int)outT), mS = (uint32_t)wv_shr1((int)outMS),
                           mL0 = (uint32_t)wv_shr1((int)outL);
            const int i = t - gl;
            const Nw16Row xr = nw16_row(xrow);
            xrow = CAREFUL ? X8[min(max(i + 1, 0), xcl)] : X8[i + 1];          // next row, read ahead
            const bool pre = PRE && i < 1;
            const bool row1 = CAREFUL && i <= 1;                     // up invalid, mc frozen (:449, :476)
            uint32_t mfS = mS, l0 = mL0;
            TbWords<K> tw = {};
#pragma unroll
            for (int s = 0; s < K; ++s) {
                const uint32_t d0 = (s == 0) ? in1 : own[s - 1];     // T[i-1][j-1]
                const uint32_t tl = (s == 0) ? sN : cur[s - 1];      // T[i][j-1]
                const uint32_t sc = nw16_sc(xr, yreg[s]);
                const uint32_t up = row1 ? NBIG : u0[s];
                const uint32_t lu = pk_maxu(l0, up);
                uint32_t v = nw16_add_sc(pk_maxu(d0, lu), sc);
                if (s == OFF) v = leadc0 ? nw16_sc_biased(sc) : v;               // column 0 (:426)
                cur[s] = pre ? own[s] : v;
                // move bits: signs of (d0 - lu) [not diagonal] and (l0 - up) [up > left] (:457-472)
                // (sign-replicating selectors 8-11: bytes 0xFF / 0x00, no shift before packing)
                const uint32_t P2 = TB ? wv_perm(pk_sub(l0, up), pk_sub(d0, lu), 0x0B0A0908u) : 0u;
                // column max of column j-1 over rows <= i-2, strict > (:476-480), in the
                // +ig+eg frame: dI[s] = T[i-2][j-1] + ig + eg; the max is the select
                const uint32_t mU = pk_neg_mask(pk_sub(mcS[s], dI[s]));
                const uint32_t u0n = wv_bfi(mU, dI[s], u0[s]) - EGN;
                u0[s] = row1 ? u0[s] : u0n;
                mcS[s] = wv_bfi(mU, dI[s], mcS[s]);
                // row state for column j+1: tested on row i, taken from row i-1 (:434-438)
                const uint32_t mnL = pk_neg_mask(pk_sub(tl, mfS));   // 0xFFFF: mf kept (not L)
                dI[s] = d0 - IGEN;                              // this row's; the next row's u2 + ig + eg
                l0 = wv_bfi(mnL, l0 - EGN, dI[s]);
                mfS = wv_bfi(mnL, mfS, d0);
                if (s == OFF) { mfS = leadc0 ? NBIG : mfS; l0 = leadc0 ? NBIG : l0; }   // j = 1: mf = T[i][0]
                if (TB) tw.add(s, P2, mU, mnL);
            }
            // rows outside [1, xlen) are never read; 32-bit byte offset from the
            // wave-uniform slot base (global_store saddr form)
            if (TB) tw.store((uint32_t *)(tb3 + ((uint32_t)(t - tb0) * RECB + (uint32_t)lane * (4u * NREC))));
            // last column (rows 1 .. xlen-2) and last row (:481-484)
            uint32_t vl = cur[LAST ? K - 1 : 0];
            if (!LAST)
#pragma unroll
                for (int s = 1; s < K; ++s) vl = wv_bfi(lastm[s], cur[s], vl);
            uint32_t km = pk_neg_mask(pk_sub(vl, bestC));             // keep where vl < best (">=" takes)
            if (CAREFUL) {
                km |= pk_neg_mask(pk_sub(limp, ipk)) | pk_neg_mask(pk_sub(ipk, pk1(1)));
                if (i >= 1 && (i == xl[0] - 1 || i == xl[1] - 1)) {
                    for (int h = 0; h < 2; ++h) {
                        if (!lact[h] || i != xl[h] - 1) continue;
#pragma unroll
                        for (int s = 0; s < K; ++s) {
                            const int j = j0 + s, val = pk_score(cur[s], h);
                            if (j >= 1 && j < yl[h] && val >= bestR[h]) { bestR[h] = val; bestRj[h] = j; }
                        }
                    }
                }
            }
            bestC = wv_bfi(km, bestC, vl);
            bestCi = wv_bfi(km, bestCi, ipk);
            ipk = pk_add(ipk, 0x10001u);
            in0 = pre ? in1 : sN;
            outT = cur[K - 1]; outMS = mfS; outL = l0;
        };
        // Checkpoint m = the state before step 1 + m*CK, where the roles
        // are (cur, own) = (A, B), (in0, in1) = (I2, I1); register r of lane l
        // at ckw[(m*NST + r)*64] (coalesced).  dI is not stored: the step
        // before a checkpoint ran with (own, in1) = (A, I2) and set dI[s] =
        // d0 - IGEN with d0 = (s ? A[s-1] : I2), neither of which it changed
        // (it wrote B and I1), so the restore recomputes it.
        constexpr bool TB1 = !TWO;                // the first sweep writes traceback only in one-pass mode
        auto save = [&](const int m) {
            uint32_t *p = ckw + (uint32_t)m * (NST * 64u);
#pragma unroll
            for (int s = 0; s < K; ++s) {
                p[s * 64] = A[s]; p[(K + s) * 64] = B[s];
                p[(2 * K + s) * 64] = mcS[s]; p[(3 * K + s) * 64] = u0[s];
            }
            p[4 * K * 64] = I1; p[(4 * K + 1) * 64] = I2;
            p[(4 * K + 2) * 64] = outT; p[(4 * K + 3) * 64] = outMS; p[(4 * K + 4) * 64] = outL;
        };
        int nextck = 1 + CK, mck = 1;
        auto ck = [&](const int t) { if (TWO && t == nextck) { save(mck); ++mck; nextck += CK; } };
        if (TWO) save(0);
        mark(0);
        // (cur, own) and (in0, in1) swap every step; every loop advances t by 2
        // so the phase carries over
        // (two-pass: steps inside the window write their traceback; t is odd
        // here, so a pair is inside or outside the window as a whole)
        auto inwin = [&](const int tt) { return TWO && tt >= tw0 && tt < tw1; };
        int t = 1;
        for (; t + 1 < tend && t <= G + 1; t += 2) {             // skewed start: lanes may be at row <= 1
            ck(t);
            if (inwin(t)) {
                step(true, true, true, t, A, B, I2, I1);
                step(true, true, true, t + 1, B, A, I1, I2);
            } else {
                step(true, true, TB1, t, A, B, I2, I1);
                step(true, true, TB1, t + 1, B, A, I1, I2);
            }
        }
        // every lane inside every record, row >= 2: before, inside and after
        // the window as three loops (one loop with a branch spills)
        auto fast = [&](const bool TBW, const int tlim) {
            for (; t + 1 <= tlim; t += 2) {
                ck(t);
                step(false, false, TBW, t, A, B, I2, I1);
                step(false, false, TBW, t + 1, B, A, I1, I2);
            }
        };
        fast(TB1, min(xmin - 2, tw0 - 1));                       // pairs ending before tw0
        if (TWO) {
            fast(true, min(xmin - 2, tw1 - 1));                  // t >= tw0 here (both odd) or past the region
            fast(false, xmin - 2);
        }
        for (; t + 1 < tend; t += 2) {
            ck(t);
            if (inwin(t)) {
                step(false, true, true, t, A, B, I2, I1);
                step(false, true, true, t + 1, B, A, I1, I2);
            } else {
                step(false, true, TB1, t, A, B, I2, I1);
                step(false, true, TB1, t + 1, B, A, I1, I2);
            }
        }
        if (t < tend) {
            if (inwin(t)) step(true, true, true, t, A, B, I2, I1);
            else          step(true, true, TB1, t, A, B, I2, I1);
        }
        wv_mem_sync();                            // traceback / checkpoints written by all lanes
        mark(1);

        // best cell per half: row-major order, ">=" -> last visited wins
        for (int h = 0; h < 2; ++h) {
            red[lane * 8 + 4 * h + 0] = bestR[h];
            red[lane * 8 + 4 * h + 1] = bestRj[h];
            red[lane * 8 + 4 * h + 2] = ownC[h] ? pk_score(bestC, h) : INT_MIN;
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
        // diagnostics (P.prof): where the best cells lie -- unpredicted (weak)
        // candidates: [6] last row, [7] last column within 40 rows of the
        // bottom (the window), [8] within 200, [9] higher; predicted ones:
        // [10] inside their window, [11] outside
        if (P.prof && in_group && gl == 0)
            for (int h = 0; h < 2; ++h) {
                if (!valid[h]) continue;
                int b;
                if (prow[h] == NW16_NOROW) {
                    const int up = xl[h] - 1 - bx[h];
                    b = up == 0 ? 6 : up <= 40 ? 7 : up <= 200 ? 8 : 9;
                } else {
                    b = (bx[h] >= prow[h] - P.win_up && bx[h] <= prow[h] + yl[h] - 1 + P.win_down) ? 10 : 11;
                }
                wv_atomic_add64(P.prof + b, 1ull);
            }
        mark(2);
        if (!TWO) {
            for (int h = 0; h < 2; ++h) {
                const TbAcc16<K, OFF> acc16 = {tbw, X8, Yp[h], gg, G, h, 0};
                nw_finish(P, acc16, xl[h], yl[h], valid[h], gg, gl, G, bscore[h], bx[h], by[h], cidx[h], sid[h]);
            }
            wv_lds_sync();
            mark(4);
            continue;
        }

        // ------------------------------------------- second sweep: the band
        // Half h restarts at step t0h[h] (a checkpoint at least band_w rows
        // above its best cell; 1 = the start) and runs until every lane of its
        // group has passed row bx[h]; per-half rows i_h = t0h[h] + tau - gl.
        bool todo[2] = {valid[0], valid[1]};
        if (tw1 > tw0) {
            // halves whose best cell (every lane's step of its row) lies in the window
            bool cov[2];
            for (int h = 0; h < 2; ++h) cov[h] = todo[h] && bx[h] + G <= tw1;
            if (wv_any(cov[0] || cov[1])) {
                for (int h = 0; h < 2; ++h) {
                    TbAcc16<K, OFF> acc16 = {tbw, X8, Yp[h], gg, G, h, tw0};
                    acc16.t1 = tw1;
                    const bool lost = nw_finish(P, acc16, xl[h], yl[h], cov[h], gg, gl, G, bscore[h], bx[h], by[h],
                                                cidx[h], sid[h]);
                    if (cov[h]) todo[h] = lost;
                    if (cov[h] && !lost && gl == 0 && in_group && P.win) wv_atomic_add(P.win, 1u);
                }
                wv_mem_sync();                    // walkers done before the second sweep overwrites the slot
            }
            mark(4);
        }
        int t0h[2] = {1, 1};
        // MASK: some half may be at row <= 1 (it restarted at step 1)
        auto step2 = [&](const bool MASK, const int tau, uint32_t (&cur)[K], const uint32_t (&own)[K],
                         uint32_t &in0, const uint32_t in1) {
            const uint32_t sN = (uint32_t)wv_shr1((int)outT), mS = (uint32_t)wv_shr1((int)outMS),
                           mL0 = (uint32_t)wv_shr1((int)outL);
            const int iA = t0h[0] + tau - gl, iB = t0h[1] + tau - gl;
            const Nw16Row xr = nw16_row(xrow);
            xrow = (X8[min(max(iA + 1, 0), xcl)] & NW16_XM_A) | (X8[min(max(iB + 1, 0), xcl)] & NW16_XM_B);
            // per-half forms of pass 1's `pre` (i < 1: row 0 repeats) and `row1` (i <= 1)
            const uint32_t pm = !MASK ? 0u : (iA < 1 ? 0x0000FFFFu : 0u) | (iB < 1 ? 0xFFFF0000u : 0u);
            const uint32_t r1 = !MASK ? 0u : (iA <= 1 ? 0x0000FFFFu : 0u) | (iB <= 1 ? 0xFFFF0000u : 0u);
            uint32_t mfS = mS, l0 = mL0;
            TbWords<K> tw = {};
#pragma unroll
            for (int s = 0; s < K; ++s) {
                const uint32_t d0 = (s == 0) ? in1 : own[s - 1];
                const uint32_t tl = (s == 0) ? sN : cur[s - 1];
                const uint32_t sc = nw16_sc(xr, yreg[s]);
                const uint32_t up = MASK ? wv_bfi(r1, NBIG, u0[s]) : u0[s];
                const uint32_t lu = pk_maxu(l0, up);
                uint32_t v = nw16_add_sc(pk_maxu(d0, lu), sc);
                if (s == OFF) v = leadc0 ? nw16_sc_biased(sc) : v;
                cur[s] = MASK ? wv_bfi(pm, own[s], v) : v;
                const uint32_t P2 = wv_perm(pk_sub(l0, up), pk_sub(d0, lu), 0x0B0A0908u);
                const uint32_t mU = pk_neg_mask(pk_sub(mcS[s], dI[s]));
                const uint32_t u0n = wv_bfi(mU, dI[s], u0[s]) - EGN;
                u0[s] = MASK ? wv_bfi(r1, u0[s], u0n) : u0n;
                mcS[s] = wv_bfi(mU, dI[s], mcS[s]);
                const uint32_t mnL = pk_neg_mask(pk_sub(tl, mfS));
                dI[s] = d0 - IGEN;
                l0 = wv_bfi(mnL, l0 - EGN, dI[s]);
                mfS = wv_bfi(mnL, mfS, d0);
                if (s == OFF) { mfS = leadc0 ? NBIG : mfS; l0 = leadc0 ? NBIG : l0; }
                tw.add(s, P2, mU, mnL);
            }
            tw.store((uint32_t *)(tb3 + ((uint32_t)tau * RECB + (uint32_t)lane * (4u * NREC))));
            in0 = MASK ? wv_bfi(pm, in1, sN) : sN;
            outT = cur[K - 1]; outMS = mfS; outL = l0;
        };
        for (int att = wv_any(todo[0] || todo[1]) ? 0 : 3; att < 3; ++att) {
            // attempt 0: the band; 1 (a path left it): NW16_BAND2 x the band;
            // 2: every half from the start
            int n2 = 0;
            for (int h = 0; h < 2; ++h) {
                const int lo = bx[h] - (att == 0 ? P.band_w : NW16_BAND2 * P.band_w) - 1;
                t0h[h] = (att < 2 && lo >= 0) ? 1 + CK * (lo / CK) : 1;
                if (todo[h]) n2 = max(n2, bx[h] + G - t0h[h]);
            }
            for (int o = 32; o > 0; o >>= 1) n2 = max(n2, wv_shfl_xor(n2, o));
            {   // restore: half A from its checkpoint, half B from its own
                const uint32_t *pa = ckw + (uint32_t)((t0h[0] - 1) / CK) * (NST * 64u);
                const uint32_t *pb = ckw + (uint32_t)((t0h[1] - 1) / CK) * (NST * 64u);
                auto ld = [&](const int r) { return wv_bfi(0x0000FFFFu, pa[r * 64], pb[r * 64]); };
#pragma unroll
                for (int s = 0; s < K; ++s) {
                    A[s] = ld(s); B[s] = ld(K + s);
                    mcS[s] = ld(2 * K + s); u0[s] = ld(3 * K + s);
                }
                I1 = ld(4 * K); I2 = ld(4 * K + 1);
                outT = ld(4 * K + 2); outMS = ld(4 * K + 3); outL = ld(4 * K + 4);
#pragma unroll
                for (int s = 0; s < K; ++s) dI[s] = (s ? A[s - 1] : I2) - IGEN;    // (save())
                xrow = (X8[min(max(t0h[0] - gl, 0), xcl)] & NW16_XM_A) | (X8[min(max(t0h[1] - gl, 0), xcl)] & NW16_XM_B);
            }
            // rows <= 1 need the masked step: while tau <= G - min(t0h) (wave-uniform bound)
            // (every half counts: one that is done still computes, and stays a bounded DP)
            int tmin = min(t0h[0], t0h[1]);
            for (int o = 32; o > 0; o >>= 1) tmin = min(tmin, wv_shfl_xor(tmin, o));
            const int tau_m = G + 1 - tmin;          // rows t0h + tau - gl > 1 for every lane from here on
            int tau = 0;
            for (; tau + 1 < n2 && tau < tau_m; tau += 2) {
                step2(true, tau, A, B, I2, I1);
                step2(true, tau + 1, B, A, I1, I2);
            }
            for (; tau + 1 < n2; tau += 2) {
                step2(false, tau, A, B, I2, I1);
                step2(false, tau + 1, B, A, I1, I2);
            }
            if (tau < n2) step2(true, tau, A, B, I2, I1);
            wv_mem_sync();                        // band traceback written by all lanes, read by the walkers
            mark(3);
            for (int h = 0; h < 2; ++h) {
                const TbAcc16<K, OFF> acc16 = {tbw, X8, Yp[h], gg, G, h, t0h[h]};
                todo[h] = nw_finish(P, acc16, xl[h], yl[h], todo[h], gg, gl, G, bscore[h], bx[h], by[h], cidx[h],
                                    sid[h]);
            }
            mark(4);
            if (!wv_any(todo[0] || todo[1])) break;
            if (lane == 0 && P.redo) wv_atomic_add(P.redo, 1u);
            wv_mem_sync();                        // walkers done before the redo overwrites the band
        }
        wv_lds_sync();
    }
    if (P.prof && lane == 0) {
        for (int k = 0; k < 5; ++k) wv_atomic_add64(P.prof + k, ph[k]);
        wv_atomic_add64(P.prof + 5, wv_realtime() - rt0);
    }
}

// Launch shape: G lanes per group, GPW groups (2*GPW candidates) per wave,
// K columns per lane
__host__ static inline NwShape nw16_shape(uint32_t ymax, uint32_t xcap, int K = NW16_K) {
    NwShape s;
    s.k = K;
    s.G = (int)((ymax + K - 1) / K);
    if (s.G < 1) s.G = 1;
    s.GPW = 64 / s.G; s.nstr = 1;
    s.xcap = xcap < 2 ? 2 : (int)xcap;
    s.xstride = (s.xcap + 15) & ~15;
    while (s.GPW > 1 && (size_t)s.GPW * s.xstride > 16384) s.GPW--;
    s.steps = s.xcap + s.G;
    return s;
}
// The 19-column form where every read of a launch has length NW16_K19_YLEN
// (150) and the shape fills the wave (imsame_dev.hip:plan_nw); on by default,
// IMSAME_NW_K19=0 (or IMSAME_NW_K=10 / 5) keeps the 10-column form.
__host__ static inline bool nw16_k19_ok(uint32_t ylen_uni, uint32_t ymax, uint32_t xcap, const imsame_params *p) {
    const char *e = getenv("IMSAME_NW_K19"), *k = getenv("IMSAME_NW_K");
    if ((e && !atoi(e)) || (k && atoi(k) != NW16_K19)) return false;
    if (ylen_uni != NW16_K19_YLEN || ymax != NW16_K19_YLEN) return false;
    if (!nw16_fits(p->igap, p->egap, xcap, ymax, NW16_K19)) return false;
    const NwShape s = nw16_shape(ymax, xcap, NW16_K19);
    return s.G * s.GPW == 64;
}
// traceback dwords per wave slot (NREC per lane per step)
__host__ static inline uint64_t nw16_tb_words(const NwShape &s) { return (uint64_t)s.steps * 64 * nw16_nrec(s.k); }
// checkpoint dwords per wave slot (two-pass mode): one per nw16_ck(K) steps + the start
__host__ static inline uint64_t nw16_ck_words(const NwShape &s) {
    return (uint64_t)((s.steps + nw16_ck(s.k) - 1) / nw16_ck(s.k) + 1) * nw16_nst(s.k) * 64;
}

#ifndef IMSAME_WAVE_EMU
// The XCD (accelerator complex die) a wave runs on: each of the 8 has its own
// L2, so an arena slot is reused only by waves of the XCD that wrote it last
// (a store that reached one L2 is not visible to, nor ordered against, the
// others until that L2 writes it back).
__device__ __forceinline__ uint32_t nw_xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v;
}
// Non-persistent launches (NwLaunch::slot_bits): a wave takes a free slot of
// its XCD's partition (lane 0 sets a bit; partitions hold the XCD's whole
// residency of the kernel, so one is always free once the wave is resident)
// and frees it when its stores have completed.  Returns ~0u only if no slot
// turned up after 2^22 probes.
__device__ uint32_t nw_slot_claim(const NwLaunch &P, const int lane) {
    const uint32_t part = nw_xcc_id() & 7u, nw = P.slot_words;
    uint32_t *bits = P.slot_bits + part * nw;
    uint32_t got = ~0u;
    if (lane == 0) {
        uint32_t w = blockIdx.x % nw;
        for (uint32_t it = 0; it < (1u << 22) && got == ~0u; ++it) {
            uint32_t v = __hip_atomic_load(bits + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            while (v != 0xFFFFFFFFu) {
                const uint32_t b = (uint32_t)__builtin_ctz(~v);
                const uint32_t old = __hip_atomic_fetch_or(bits + w, 1u << b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (!(old & (1u << b))) { got = (part * nw + w) * 32u + b; break; }
                v = old | (1u << b);
            }
            if (got == ~0u && ++w == nw) { w = 0; __builtin_amdgcn_s_sleep(4); }
        }
    }
    got = __builtin_amdgcn_readfirstlane(wv_shfl((int)got, 0));
    // The slot's last user may have run on another CU of this XCD: this CU's
    // vector L1 can still hold lines of the slot from an earlier user here
    // (L1 is invalidated at kernel starts, not when a slot changes hands
    // inside a launch), so drop them before the first access.
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    return got;
}
__device__ __forceinline__ void nw_slot_release(const NwLaunch &P, const int lane, const uint32_t slot) {
    __builtin_amdgcn_s_waitcnt(0);                 // every store of this wave has reached the XCD's L2
    if (lane == 0)
        __hip_atomic_fetch_and(P.slot_bits + (slot >> 5), ~(1u << (slot & 31u)), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
}

// XCC_ID of every block (imsame_dev.hip checks it before it trusts the
// partitions above)
__global__ void xcc_probe_kernel(uint32_t *out) {
    if (threadIdx.x == 0) out[blockIdx.x] = nw_xcc_id();
}

// 3 waves per SIMD (168 VGPRs): at 4 (128) the compiler spills in the sweep
// loops; the first-sweep loop issues 3.81 vs 3.95 cycles per VALU per SIMD
// (scripts/micro/nw16_loop.py, profiles/r4c/) and C2 runs 1.5 % faster
// (profiles/r4c/benchab_*)
#ifndef NW16_WAVES_PER_EU
#define NW16_WAVES_PER_EU 3
#endif
#ifndef NW16_K5_WAVES_PER_EU
#define NW16_K5_WAVES_PER_EU 5
#endif
// (K = 3: 4 waves per SIMD, 128 VGPRs -- at 5 its second-sweep loops spill;
// its launches are latency-bound, a few waves per SIMD.  The context's slot
// partitions hold the largest residency of any packed form, nw16_np_part_cu)
#ifndef NW16_K3_WAVES_PER_EU
#define NW16_K3_WAVES_PER_EU 4
#endif
// the 19-column form holds 6 x 19 per-column registers: 2 waves per SIMD (256
// VGPRs), which the first-sweep loop's ILP keeps issuing (a 2-wave SIMD ran
// the 10-column loop at 4.0 cycles per VALU, profiles/r4b/micro_*)
#ifndef NW16_K19_WAVES_PER_EU
#define NW16_K19_WAVES_PER_EU 2
#endif
template <int K, bool LAST, bool TWO, int OFF = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(K > 10 ? NW16_K19_WAVES_PER_EU
                                                                     : K > 8 ? NW16_WAVES_PER_EU
                                                                     : K > 3 ? NW16_K5_WAVES_PER_EU
                                                                             : NW16_K3_WAVES_PER_EU)))
void nw16_kernel(NwLaunch P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    // One call site, so nw16_wave is inlined: with two (persistent and
    // non-persistent) the compiler outlined it as a function, 3 % slower at
    // C2 (profiles/r3v_*: 127.1 vs 123.3 ms per step on one box).
    uint32_t slot;
    if (P.slot_bits) {                          // non-persistent: one task, a slot of this XCD
        slot = nw_slot_claim(P, lane);
        if (slot == ~0u) {                      // never (partitions hold the residency).  This wave's
            if (lane == 0) wv_atomic_or(P.flags, 4u);     // task is NOT run by anyone: the flag makes the
            return;                             // update_kernel behind the launch consume nothing and
        }                                       // the host fail the call (align_one)
    } else {
        slot = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + wib);   // wave-uniform
    }
    nw16_wave<K, LAST, TWO, OFF>(P, smem + wib * nw16_wave_lds(P.GPW, P.xstride), lane, slot);
    if (P.slot_bits) nw_slot_release(P, lane, slot);
}
#endif
