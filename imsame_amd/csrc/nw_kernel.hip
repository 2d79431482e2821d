// nw_kernel.hip -- IMSAME's gapped "NW" + backtracking as an anti-diagonal
// wavefront on gfx950 wave64.  Included by imsame_dev.hip (and, for the CPU
// test suite, by tests/emu/wave_emu.cpp under IMSAME_WAVE_EMU).
//
// Reference: NW              alignmentFunctions.c:389-489
//            backtrackingNW  alignmentFunctions.c:493-560
//            identities      alignmentFunctions.c:254-265 (build_alignment)
//            acceptance      alignmentFunctions.c:163
//
// Mapping.  One candidate (X = database record: rows i, Y = read: columns j)
// is a GROUP of G lanes; lane gl owns NW_K consecutive columns of a strip of
// NW_W = 64*NW_K columns and walks the rows with a one-step skew: at step t
// lane gl computes row i = t - gl.  The row state of IMSAME's recurrence
// ("mf", the lagged running row maximum) flows lane -> lane+1 through a DPP
// wave_shr:1; the column state ("mc[j-1]", max of column j-1 over rows
// <= i-3) is lane-local.  64/G candidates share a wave (G = ceil(ylen/NW_K)).
// Reads longer than NW_W/2 use one group per wave and several strips, the
// strip seam (T[i][c], mf) passing through a per-wave global buffer.
//
// Traceback: 4 bits per cell, the 5 cells of a lane packed in one dword, so a
// step is one coalesced 256-byte wave store (0.8 B/cell):
//     bits 0-1  move: 0 diagonal, 1 up (jump from mc[j-1]), 2 left (from mf)
//     bit  2    U: mc[j-1] took (T[i-2][j-1], row i-2) at this cell (:476-480)
//     bit  3    L: mf took (T[i-1][j-1], col j-1) after this cell (:434-438)
// A jump's source is recovered in the walk: an up move at (i,j) comes from
// row (last U of column j above i) - 2 (row 0 if none); a left move from
// column (last L of row i left of j) - 1.  Identities are X[i]==Y[j] on the
// diagonal steps (:254-265).  The walk reads G cells per step (ballots find
// the first jump / the last U or L bit).
// Scores are int32: the host rejects gap parameters whose score range could
// leave +-2^26 (IMSAME_E_RANGE); NW_BIG = 2^28 stands for INT64_MIN.
#include "wave_ops.h"

#define NW_K   5                  // columns per lane
#define NW_W   (64 * NW_K)        // columns per strip
#define NW_BIG (1 << 28)

struct NwLaunch {
    const uint8_t  *db;  const uint64_t *db_start;    // db_start[n_db] = db_len
    const uint8_t  *q;   const uint64_t *q_start;     // q_start[n_q]  = q_len
    const uint32_t *cand_read, *cand_sid;
    uint32_t n_cand;
    // nw16 two-pass: optional work order (slot w of the queue takes candidate
    // perm[w]) and each candidate's predicted first row (the seed hit's
    // diagonal, NW16_NOROW = none), see nw16_kernel.hip
    const uint32_t *perm; const int32_t *cand_row;
    uint32_t *win;               // count of candidates walked inside their first-sweep window
    int32_t  win_up, win_down;   // window rows above / below the predicted ones
    int32_t  win_bottom;         // unpredicted candidate: its last rows (< 0: no window)
    int32_t  igap, egap;
    int32_t  G, GPW;             // lanes per group, groups per wave
    int32_t  xcap;               // max xlen of the launch
    int32_t  xstride;            // LDS bytes per group for X (xcap rounded up)
    int32_t  steps;              // traceback steps per strip (xcap + G)
    uint32_t *tb;                // traceback scratch, one slot per resident wave
    uint64_t tb_wave_dw;         // dwords per slot
    int32_t  *bnd;               // strip seam scratch, one slot per resident wave
    uint64_t bnd_wave;           // ints per slot (3 * xcap)
    const uint32_t *minlen;      // [ylen]  minimum length for coverage
    const uint32_t *minident;    // [len]   minimum identities for identity
    uint32_t n_minlen, n_minident;
    uint32_t *counter;           // work queue head
    imsame_read_result *out;     // per candidate
    uint32_t *paths; uint32_t paths_cap; uint32_t *paths_used; uint32_t want_paths;
    uint32_t *flags;             // bit0: path arena overflow, bit1: walk guard tripped
    // nw16 two-pass mode (nw16_kernel.hip): checkpoints of the first sweep,
    // one slot per resident wave; rows above a best cell the band keeps;
    // count of waves whose band missed a path (second sweep redone from row 1)
    uint32_t *ck; uint64_t ck_wave_dw;
    int32_t  band_w;
    uint32_t *redo;
    unsigned long long *prof;    // optional (IMSAME_NW_PROF): shader cycles per phase, summed over waves
    // non-persistent launches (nw16_kernel): one wave per task, its arena slot
    // taken from a bitmap of free slots in the partition of the XCD it runs on
    // (NULL: persistent launch, slot = the wave's index in the grid)
    uint32_t *slot_bits; uint32_t slot_words;   // words per XCD partition
    // packed long-read kernel (nwp_kernel.hip): |ig| + |eg| (L + 64) of the
    // launch (nwp_fits), the T spread checked every block, and the count of
    // waves that found a value outside the proof's range (their pairs ran
    // through the int32 nwl_cand instead)
    int32_t rlim, nwp_s;
    uint32_t *fbk;
};

// LDS bytes one wave needs
__host__ __device__ static inline size_t nw_wave_lds(int GPW, int xstride) { return (size_t)GPW * xstride + 64 * 16; }

// dword index of (strip st, step t, wave lane wl)
__device__ __forceinline__ uint32_t tb_word(int st, int t, int wl, int steps) {
    return ((uint32_t)st * steps + t) * 64u + wl;
}
// nibble of cell (i, j) of group g
__device__ __forceinline__ uint32_t tb_cell(const uint32_t *tb, int i, int j, int g, int G, int steps) {
    const int st = j / NW_W, jj = j - st * NW_W, l = jj / NW_K, s = jj - l * NW_K;
    return (tb[tb_word(st, i + l, g * G + l, steps)] >> (4 * s)) & 0xFu;
}

// per-candidate constants of one group, as seen by one lane
struct NwCand {
    const uint8_t *X;      // LDS copy of the record
    const uint8_t *Y;      // read in global memory
    int xlen, ylen;
};

// The sweep of one strip: rows 1 .. xlen-1 of this lane's NW_K columns.
// SEAM_IN: the strip's lead lane takes its left neighbour from the seam
// buffer; SEAM_OUT: the strip's last lane writes its right edge there.
template <bool SEAM_IN, bool SEAM_OUT>
__device__ __forceinline__ void nw_sweep(const NwLaunch &P, const NwCand &cd, uint32_t *tbw, int *bnd, const int st,
                                         const int lane, const int gl, const int G, const int xmax, const bool cvalid,
                                         int &bestR, int &bestRj, int &bestC, int &bestCi) {
    const int ig = P.igap, eg = P.egap;
    const int xlen = cd.xlen, ylen = cd.ylen;
    const int xl1 = xlen > 1 ? xlen - 1 : 1;
    const int j0 = st * NW_W + gl * NW_K;
    const bool lact = cvalid && j0 < ylen;
    const bool leadc0 = (gl == 0) && st == 0;
    const bool lead_seam = SEAM_IN && gl == 0;
    const bool seam_out = SEAM_OUT && (gl == G - 1) && cvalid;
    const int lastj = ylen - 1;
    const bool owns_last = cvalid && lastj >= j0 && lastj < j0 + NW_K;
    const int s_last = lastj - j0;
    int Y[NW_K], cJ[NW_K], colc[NW_K];
#pragma unroll
    for (int s = 0; s < NW_K; ++s) {
        const int j = j0 + s;
        Y[s] = (cvalid && j < ylen) ? (int)cd.Y[j] : 0;
        cJ[s] = (j <= 1) ? -NW_BIG : ig + (j - 1) * eg;        // left needs j > 1 (:443)
        colc[s] = -eg * (j - 1);
    }
    // row 0 (:404-413): T[0][j] = s(X0,Yj); mc[j] = (T[0][j], row 0)
    const int x0 = cvalid ? (int)cd.X[0] : 0;
    // (a lane wholly past the read's end computes garbage columns only: it must
    // not read past the read -- found by the ASan build of the emulator)
    const int yprev = (cvalid && j0 > 0 && j0 <= ylen) ? (int)cd.Y[j0 - 1] : 0;
    const int t0prev = (x0 == yprev) ? 4 : -4;
    // Three rotating row buffers (cur / own = row i-1 / own2 = row i-2), all
    // starting as row 0.  A lane repeats row 0 until its first row and runs
    // past its last row with bounded garbage nobody reads, so every step is
    // branch-free; row 0 standing in for row -1 cannot trigger an mc update
    // (T[0][j-1] is not > mc[j-1] = T[0][j-1]).
    int A[NW_K], B[NW_K], C[NW_K], mcS[NW_K], mcAdj[NW_K];
#pragma unroll
    for (int s = 0; s < NW_K; ++s) { A[s] = (x0 == Y[s]) ? 4 : -4; B[s] = A[s]; C[s] = A[s]; }
#pragma unroll
    for (int s = 0; s < NW_K; ++s) {
        mcS[s] = (s == 0) ? t0prev : A[s - 1];
        mcAdj[s] = mcS[s];
        if (j0 + s == 1) mcS[s] = NW_BIG;          // mc[0] is never updated (j > 1 test, :476)
    }
    int I1 = t0prev, I2 = t0prev, I3 = t0prev;     // left neighbour's column, rotating like A/B/C
    // row state crossing lanes: (T[i][c], mf score, mf score - egap * mf column)
    int outT = A[NW_K - 1], outMS = 0, outMA = 0;
    const int tend = xmax - 1 + G;
    int xnext = (int)cd.X[min(max(1 - gl, 0), xl1)];
    int bnext0 = 0, bnext1 = 0, bnext2 = 0;
    if (lead_seam && cvalid) { bnext0 = bnd[3]; bnext1 = bnd[4]; bnext2 = bnd[5]; }

    // PRE: some lane may still be before its first row (t <= G); constant at every call
    auto step = [&](const bool PRE, const int t, int (&cur)[NW_K], const int (&own)[NW_K], const int (&own2)[NW_K],
                    int &in0, const int in1, const int in2) {
        int sN = wv_shr1(outT), mS = wv_shr1(outMS), mA = wv_shr1(outMA);
        const int i = t - gl;
        const int xi = xnext;
        xnext = (int)cd.X[min(max(i + 1, 0), xl1)];                    // next step's row, read ahead
        if (SEAM_IN) {
            if (lead_seam) { sN = bnext0; mS = bnext1; mA = bnext2; }
            const int ni = min(max(i + 1, 1), xl1);
            if (lead_seam && cvalid) { bnext0 = bnd[3 * ni]; bnext1 = bnd[3 * ni + 1]; bnext2 = bnd[3 * ni + 2]; }
        }
        const bool pre = PRE && i < 1;
        const int cI = (i <= 1) ? -NW_BIG : ig + (i - 1) * eg;        // up needs i > 1 (:449)
        const int rowc2 = -eg * (i - 2);
        int mfS = mS, mfAdj = mA;
        uint32_t word = 0;
#pragma unroll
        for (int s = 0; s < NW_K; ++s) {
            const int d0 = (s == 0) ? in1 : own[s - 1];     // T[i-1][j-1]
            const int u2 = (s == 0) ? in2 : own2[s - 1];    // T[i-2][j-1]
            const int tl = (s == 0) ? sN : cur[s - 1];      // T[i][j-1]
            const bool m = xi == Y[s];
            const int l0 = mfAdj + cJ[s];                   // left - s  (:444)
            const int u0 = mcAdj[s] + cI;                   // up   - s  (:450)
            const int mx = wv_max3(d0, l0, u0);
            int v = mx + (m ? 4 : -4);
            // diag if >= both, else up if up > left, else left (:457-472)
            const uint32_t mv = (mx == d0) ? 0u : ((u0 > l0) ? 1u : 2u);
            if (s == 0) v = leadc0 ? (m ? 4 : -4) : v;       // column 0 (:426)
            cur[s] = pre ? own[s] : v;
            // column max of column j-1 over rows <= i-2, strict > (:476-480)
            const bool cu = u2 > mcS[s];
            mcAdj[s] = cu ? u2 + rowc2 : mcAdj[s];
            mcS[s] = max(mcS[s], u2);
            // row state for column j+1: tested on row i, taken from row i-1 (:434-438)
            const bool cl = mfS <= tl;
            mfAdj = cl ? d0 + colc[s] : mfAdj;             // mf - egap * (j - 1)
            mfS = cl ? d0 : mfS;
            if (s == 0) mfS = leadc0 ? -NW_BIG : mfS;        // then mf = T[i-1][0]
            word |= (mv | (cu ? 4u : 0u) | (cl ? 8u : 0u)) << (4 * s);
        }
        tbw[tb_word(st, t, lane, P.steps)] = word;          // rows outside [1, xlen) are never read
        if (lact && i == xlen - 1) {                         // last row (:481)
#pragma unroll
            for (int s = 0; s < NW_K; ++s) {
                const int j = j0 + s;
                if (j >= 1 && j < ylen && cur[s] >= bestR) { bestR = cur[s]; bestRj = j; }
            }
        }
        {                                                    // last column, rows 1 .. xlen-2
            int v = cur[0];
#pragma unroll
            for (int s = 1; s < NW_K; ++s) v = (s_last == s) ? cur[s] : v;
            const bool up = owns_last && i >= 1 && i < xlen - 1 && v >= bestC;
            bestC = up ? v : bestC;
            bestCi = up ? i : bestCi;
        }
        in0 = pre ? in1 : sN;
        outT = cur[NW_K - 1]; outMS = mfS; outMA = mfAdj;
        if (seam_out && i >= 1 && i < xlen) { bnd[3 * i] = outT; bnd[3 * i + 1] = mfS; bnd[3 * i + 2] = mfAdj; }
    };
    // roles (cur, own, own2) and (in0 <- T[i][c], in1 = T[i-1][c], in2 = T[i-2][c]) rotate every step
    int t = 1;
    for (; t + 2 < tend && t <= G; t += 3) {      // skewed start: lanes may be before row 1
        step(true, t, A, B, C, I3, I1, I2);
        step(true, t + 1, C, A, B, I2, I3, I1);
        step(true, t + 2, B, C, A, I1, I2, I3);
    }
    for (; t + 2 < tend; t += 3) {
        step(false, t, A, B, C, I3, I1, I2);       // A = row i,   B = i-1, C = i-2
        step(false, t + 1, C, A, B, I2, I3, I1);   // C = row i+1, A = i,   B = i-1
        step(false, t + 2, B, C, A, I1, I2, I3);   // B = row i+2, C = i+1, A = i
    }
    if (t < tend) step(true, t, A, B, C, I3, I1, I2);
    if (t + 1 < tend) step(true, t + 1, C, A, B, I2, I3, I1);
}

// Walk the traceback of group g from (px,py) (backtrackingNW, :493-560).
// Returns path statistics; emits runs into `path` when emit (lane gl == 0).
// TB gives nib(i, j) -- the cell's nibble in the layout above -- and
// match(i, j) = X[i] == Y[j]; one accessor per traceback layout.
// lost: the path needs a cell the traceback does not hold (TB::has false --
// the nw16 second sweep's band); the caller recomputes and walks again.
struct WalkOut { int len, idn, ig, eg, cx, cy, nent; bool bad, lost; };

struct TbAcc32 {                       // this file's layout: one candidate per group
    const uint32_t *tb; const NwCand *cd; int g, G, steps;
    __device__ bool has(int, int) const { return true; }
    __device__ uint32_t nib(int i, int j) const { return tb_cell(tb, i, j, g, G, steps); }
    __device__ bool match(int i, int j) const { return cd->X[i] == cd->Y[j]; }
};

template <class TB>
__device__ WalkOut nw_walk(const TB &tbk, int xlen, int ylen, int px, int py, bool walking, int g, int gl,
                           int G, uint32_t *path, bool emit) {
    WalkOut w = {0, 0, 0, 0, px, py, 0, false, false};
    const unsigned long long gmask = (G == 64) ? ~0ull : ((1ull << G) - 1);
    int run = 0;                       // pending diagonal run (emit) / in-run flag
    int guard = 4 * (xlen + ylen) + 8;
    walking = walking && px > 0 && py > 0;
    while (wv_any(walking)) {
        // G diagonal cells at once; the first non-diagonal one stops the run
        const int cx = px - gl, cy = py - gl;
        const bool valid = walking && cx >= 1 && cy >= 1;
        const bool av = valid && tbk.has(cx, cy);
        uint32_t nib = 0xFu;
        bool match = false;
        if (av) {
            nib = tbk.nib(cx, cy);
            match = tbk.match(cx, cy);
        }
        const bool stop = !av || (nib & 3u) != 0;
        const unsigned long long bs = wv_ballot(stop), bm = wv_ballot(av && match);
        const unsigned long long bl = (wv_ballot(valid && !av) >> (g * G)) & gmask;
        const unsigned long long gs = (bs >> (g * G)) & gmask;
        const int first = gs ? __builtin_ctzll(gs) : G;
        const unsigned long long below = (first >= 64) ? ~0ull : ((1ull << first) - 1);
        const int nm = __builtin_popcountll((bm >> (g * G)) & gmask & below);
        const uint32_t mvj = (uint32_t)wv_shfl((int)(nib & 3u), g * G + (first < G ? first : 0));
        if (walking) {
            if (first > 0) {
                if (!run) w.nent++;
                if (emit) run += first; else run = 1;
                w.len += first; w.idn += nm; px -= first; py -= first;
            }
            if (first < G && ((bl >> first) & 1ull)) { w.lost = true; walking = false; }   // stopped at a missing cell
        }
        const bool jump = walking && first < G && px > 0 && py > 0;
        if (walking && jump && (mvj == 0u || mvj == 3u)) { w.bad = true; walking = false; }
        // up: last row i < px of column py with U set -> source row i-2 (0 if none)
        const bool want_up = wv_any(jump && !w.bad && mvj == 1u);
        const bool want_left = wv_any(jump && !w.bad && mvj == 2u);
        int src = 0;
        bool is_up = jump && mvj == 1u, is_left = jump && mvj == 2u;
        if (want_up) {
            bool searching = is_up;
            int base = px - 1;
            src = 0;
            while (wv_any(searching)) {
                const int r = base - gl;
                const bool ok = searching && r >= 1;
                const bool av = ok && tbk.has(r, py);
                const bool u = av && ((tbk.nib(r, py) >> 2) & 1u);
                const unsigned long long gb = (wv_ballot(u) >> (g * G)) & gmask;
                const unsigned long long gm = (wv_ballot(ok && !av) >> (g * G)) & gmask;
                if (searching) {
                    // a missing row above (before) the first U found: the U may be there
                    if (gm && (!gb || __builtin_ctzll(gm) < __builtin_ctzll(gb))) { w.lost = true; searching = false; }
                    else if (gb) { src = base - __builtin_ctzll(gb) - 2; searching = false; }
                    else if (base - G < 1) { src = 0; searching = false; }
                    else base -= G;
                }
            }
        }
        if (want_left) {
            bool searching = is_left;
            int base = py - 1;
            int lsrc = 0;
            while (wv_any(searching)) {
                const int c = base - gl;
                const bool ok = searching && c >= 1;
                const bool av = ok && tbk.has(px, c);
                const bool l = av && ((tbk.nib(px, c) >> 3) & 1u);
                const unsigned long long gb = (wv_ballot(l) >> (g * G)) & gmask;
                const unsigned long long gm = (wv_ballot(ok && !av) >> (g * G)) & gmask;
                if (searching) {
                    if (gm && (!gb || __builtin_ctzll(gm) < __builtin_ctzll(gb))) { w.lost = true; searching = false; }
                    else if (gb) { lsrc = base - __builtin_ctzll(gb) - 1; searching = false; }
                    else if (base - G < 1) { w.bad = true; searching = false; }   // L(i,1) always set
                    else base -= G;
                }
            }
            if (is_left) src = lsrc;
        }
        if (w.lost) walking = false;
        if (walking && jump && !w.bad) {
            int n;
            if (is_up) { n = px - src; px = src; py -= 1; }     // X run vs '-'  (:520-530)
            else       { n = py - src; py = src; px -= 1; }     // '-' vs Y run  (:531-543)
            if (n < 1) { w.bad = true; walking = false; }
            if (emit && gl == 0 && !w.bad) {
                if (run) path[w.nent - 1] = (IMSAME_MOVE_DIAG << 30) | (uint32_t)run;
                path[w.nent] = ((is_up ? IMSAME_MOVE_UP : IMSAME_MOVE_LEFT) << 30) | (uint32_t)n;
            }
            w.nent++;
            run = 0;
            w.len += n; w.eg += n - 1; w.ig += 1;
        }
        if (w.bad) walking = false;
        if (walking) {
            walking = px > 0 && py > 0;
            if (--guard < 0) { w.bad = true; walking = false; }
        }
    }
    if (emit && gl == 0 && run && !w.bad && !w.lost) path[w.nent - 1] = (IMSAME_MOVE_DIAG << 30) | (uint32_t)run;
    w.cx = px; w.cy = py;
    return w;
}

// Backtrack + acceptance + result of one candidate per group (all lanes of
// the wave call it; lanes with !cvalid only take part in the wave votes).
// Returns true (and writes nothing) where the path left the traceback held.
template <class TB>
__device__ bool nw_finish(const NwLaunch &P, const TB &acc32, const int xlen, const int ylen, const bool cvalid0,
                          const int gg, const int gl, const int G, const int bscore, const int bx, const int by,
                          const uint32_t c, const uint32_t sid) {
        WalkOut w = nw_walk(acc32, xlen, ylen, bx, by, cvalid0, gg, gl, G, nullptr, false);
        const bool lost = cvalid0 && w.lost;
        const bool cvalid = cvalid0 && !w.lost;
        bool acc = false;
        if (cvalid && !w.bad) {
            acc = (uint32_t)ylen < P.n_minlen && (uint32_t)w.len >= P.minlen[ylen] &&
                  (uint32_t)w.len < P.n_minident && (uint32_t)w.idn >= P.minident[w.len];
        }
        if (cvalid && w.bad && gl == 0) wv_atomic_or(P.flags, 2u);
        uint32_t poff = 0, plen = 0;
        const bool want = cvalid && acc && P.want_paths;
        if (wv_any(want)) {
            uint32_t off = 0;
            if (want && gl == 0) {
                off = wv_atomic_add(P.paths_used, (uint32_t)w.nent);
                if (off + (uint32_t)w.nent > P.paths_cap) { wv_atomic_or(P.flags, 1u); off = 0xFFFFFFFFu; }
            }
            off = (uint32_t)wv_shfl((int)off, gg * G);
            const bool ok = want && off != 0xFFFFFFFFu;
            nw_walk(acc32, xlen, ylen, bx, by, ok, gg, gl, G, ok ? P.paths + off : nullptr, true);
            if (ok) { poff = off; plen = (uint32_t)w.nent; }
            // arena full: the path is LOST (path_off ~0) and path_len says how
            // many entries it needs; the host re-walks exactly these pairs
            else if (want) { poff = 0xFFFFFFFFu; plen = (uint32_t)w.nent; }
        }
        if (cvalid && gl == 0) {
            const int M = 2 * max(xlen, ylen);
            const int tail = w.cx + w.cy;                    // one of them is 0
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
        return lost;
}

// One wave's share of a launch: pulls groups of GPW candidates from the work
// queue until it is empty.  wsm = this wave's LDS (nw_wave_lds bytes).
// MULTI: the launch holds reads longer than one strip (one group per wave).
template <bool MULTI>
__device__ void nw_wave(const NwLaunch &P, uint8_t *wsm, const int lane, const uint32_t slot) {
    const int G = P.G, GPW = P.GPW;
    const int g = lane / G, gl = lane - g * G;
    const bool in_group = g < GPW;
    const int gg = in_group ? g : 0;
    int *red = (int *)(wsm + GPW * P.xstride);                      // 64 x 4 ints
    uint32_t *tbw = P.tb + (uint64_t)slot * P.tb_wave_dw;
    int *bnd = P.bnd + (uint64_t)slot * P.bnd_wave;

    for (;;) {
        uint32_t base = 0;
        if (lane == 0) base = wv_atomic_add(P.counter, (uint32_t)GPW);
        base = wv_first(base);
        if (base >= P.n_cand) break;
        const uint32_t c = base + g;
        const bool cvalid = in_group && c < P.n_cand;
        NwCand cd;
        cd.X = wsm + gg * P.xstride;
        cd.Y = P.q;
        cd.xlen = 0; cd.ylen = 0;
        uint64_t xo = 0;
        uint32_t sid = 0;
        if (cvalid) {
            const uint32_t rd = P.cand_read[c];
            sid = P.cand_sid[c];
            xo = P.db_start[sid]; cd.xlen = (int)(P.db_start[sid + 1] - xo);
            const uint64_t yo = P.q_start[rd];
            cd.Y = P.q + yo; cd.ylen = (int)(P.q_start[rd + 1] - yo);
        }
        if (cvalid)
            for (int k = gl; k < cd.xlen; k += G) ((uint8_t *)cd.X)[k] = P.db[xo + k];
        wv_lds_sync();

        int xmax = cd.xlen, nstr = cvalid ? (cd.ylen + NW_W - 1) / NW_W : 0;
        for (int o = 32; o > 0; o >>= 1) {
            xmax = max(xmax, wv_shfl_xor(xmax, o));
            nstr = max(nstr, wv_shfl_xor(nstr, o));
        }
        int bestR = INT_MIN, bestRj = 0, bestC = INT_MIN, bestCi = 0;
        if (!MULTI) {
            nw_sweep<false, false>(P, cd, tbw, bnd, 0, lane, gl, G, xmax, cvalid, bestR, bestRj, bestC, bestCi);
        } else {
            for (int st = 0; st < nstr; ++st) {
                // a read of one strip in a multi-strip launch has no seam at all
                // (its lead lane is column 0: reading the seam buffer there took
                // whatever an earlier candidate or allocation left in it)
                const bool in = st > 0, outs = st + 1 < nstr;
                if (!in && outs)
                    nw_sweep<false, true>(P, cd, tbw, bnd, st, lane, gl, G, xmax, cvalid, bestR, bestRj, bestC, bestCi);
                else if (in && outs)
                    nw_sweep<true, true>(P, cd, tbw, bnd, st, lane, gl, G, xmax, cvalid, bestR, bestRj, bestC, bestCi);
                else if (in)
                    nw_sweep<true, false>(P, cd, tbw, bnd, st, lane, gl, G, xmax, cvalid, bestR, bestRj, bestC, bestCi);
                else
                    nw_sweep<false, false>(P, cd, tbw, bnd, st, lane, gl, G, xmax, cvalid, bestR, bestRj, bestC, bestCi);
                wv_mem_sync();                    // seam written by the last lane, read by the lead
            }
        }
        wv_mem_sync();                            // traceback written by all lanes, read by the walkers

        // best cell (:481-484): row-major order, ">=" -> last visited wins:
        // last-row cells (largest j) beat last-column cells (largest i).
        red[lane * 4 + 0] = bestR; red[lane * 4 + 1] = bestRj;
        red[lane * 4 + 2] = bestC; red[lane * 4 + 3] = bestCi;
        wv_lds_sync();
        int bR = INT_MIN, bRj = 0, bC = INT_MIN, bCi = 0;
        if (in_group)
            for (int k = 0; k < G; ++k) {
                const int *e = red + (g * G + k) * 4;
                if (e[0] > bR || (e[0] == bR && e[1] > bRj)) { bR = e[0]; bRj = e[1]; }
                if (e[2] > bC || (e[2] == bC && e[3] > bCi)) { bC = e[2]; bCi = e[3]; }
            }
        int bscore, bx, by;
        if (bR >= bC) { bscore = bR; bx = cd.xlen - 1; by = bRj; }
        else          { bscore = bC; bx = bCi; by = cd.ylen - 1; }
        wv_lds_sync();

        const TbAcc32 acc32 = {tbw, &cd, gg, G, P.steps};
        nw_finish(P, acc32, cd.xlen, cd.ylen, cvalid, gg, gl, G, bscore, bx, by, c, sid);
        wv_lds_sync();
    }
}

// Launch shape for reads up to ymax and records up to xcap: short reads pack
// 64/G candidates per wave, long reads take a wave each over several strips;
// X staging is capped at 16 KB of LDS per wave.
struct NwShape { int G, GPW, nstr, xcap, xstride, steps, k = 0; };   // k: nw16 columns per lane
__host__ static inline NwShape nw_shape(uint32_t ymax, uint32_t xcap) {
    NwShape s;
    if (ymax <= NW_W / 2) {
        s.G = (int)((ymax + NW_K - 1) / NW_K);
        if (s.G < 1) s.G = 1;
        s.GPW = 64 / s.G; s.nstr = 1;
    } else {
        s.G = 64; s.GPW = 1; s.nstr = (int)((ymax + NW_W - 1) / NW_W);
    }
    s.xcap = xcap < 2 ? 2 : (int)xcap;
    s.xstride = (s.xcap + 15) & ~15;
    while (s.GPW > 1 && (size_t)s.GPW * s.xstride > 16384) s.GPW--;
    s.steps = s.xcap + s.G;
    return s;
}
// traceback dwords per wave slot
__host__ static inline uint64_t nw_tb_words(const NwShape &s) { return (uint64_t)s.nstr * s.steps * 64; }

#ifndef IMSAME_WAVE_EMU
// Waves per SIMD the register budget is cut for (4 = 128 VGPRs: the sweep
// loop fits without spills; the few spills land outside it).
#ifndef NW_WAVES_PER_EU
#define NW_WAVES_PER_EU 4
#endif
template <bool MULTI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MULTI ? 3 : NW_WAVES_PER_EU)))
void nw_kernel(NwLaunch P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    const uint32_t slot = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + wib);   // wave-uniform
    nw_wave<MULTI>(P, smem + wib * nw_wave_lds(P.GPW, P.xstride), lane, slot);
}
#endif
