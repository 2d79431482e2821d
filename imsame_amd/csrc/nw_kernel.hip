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
// Per cell one 16-bit traceback code is stored (skewed layout -> every step
// is one contiguous 768-byte wave store):
//     diagonal : 0 / 1 (1 = X[i]==Y[j], the identity bit)
//     up       : 0x8000 | source row   (jump from mc[j-1], column j-1)
//     left     : 0xC000 | source col   (jump from mf, row i-1)
// After the sweep each group walks its path from the best cell with
// G-wide speculative diagonal reads (ballot on the first non-diagonal code).
// Scores are int32: the host rejects gap parameters whose score range could
// leave +-2^26 (IMSAME_E_RANGE); NW_BIG = 2^28 stands for INT64_MIN.
#include "wave_ops.h"

#define NW_K   5                  // columns per lane
#define NW_KW  3                  // dwords of traceback per lane per step
#define NW_W   (64 * NW_K)        // columns per strip
#define NW_BIG (1 << 28)

struct NwLaunch {
    const uint8_t  *db;  const uint64_t *db_start;    // db_start[n_db] = db_len
    const uint8_t  *q;   const uint64_t *q_start;     // q_start[n_q]  = q_len
    const uint32_t *cand_read, *cand_sid;
    uint32_t n_cand;
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
};

// LDS bytes one wave needs
__host__ __device__ static inline size_t nw_wave_lds(int GPW, int xstride) { return (size_t)GPW * xstride + 64 * 16; }

__device__ __forceinline__ uint32_t tb_index(int st, int t, int wl, int s, int steps) {
    // u16 index of (strip st, step t, wave lane wl, sub-column s)
    return ((((uint32_t)st * steps + t) * 64u + wl) * NW_KW + (s >> 1)) * 2u + (s & 1);
}

// Walk the traceback of group g from (px,py).  Returns path statistics;
// emits runs into `path` when emit (lane gl == 0 writes).
struct WalkOut { int len, idn, ig, eg, cx, cy, nent; bool bad; };

__device__ WalkOut nw_walk(const uint16_t *tb16, int px, int py, bool walking, int g, int gl, int G,
                           int steps, uint32_t *path, bool emit) {
    WalkOut w = {0, 0, 0, 0, px, py, 0, false};
    const unsigned long long gmask = (G == 64) ? ~0ull : ((1ull << G) - 1);
    int run = 0;                       // pending diagonal run (emit) / in-run flag
    int guard = px + py + 4;           // every iteration moves at least one cell
    walking = walking && px > 0 && py > 0;
    while (wv_any(walking)) {
        const int cx = px - gl, cy = py - gl;
        const bool valid = walking && cx >= 1 && cy >= 1;
        uint32_t code = 0xFFFFu;
        if (valid) {
            const int st = cy / NW_W, jj = cy - st * NW_W, l = jj / NW_K, s = jj - l * NW_K;
            code = tb16[tb_index(st, cx + l, g * G + l, s, steps)];
        }
        const bool stop = !valid || (code >> 14) != 0;
        const unsigned long long bs = wv_ballot(stop), bmatch = wv_ballot(valid && code == 1u);
        const unsigned long long gs = (bs >> (g * G)) & gmask;
        const int first = gs ? __builtin_ctzll(gs) : G;
        const unsigned long long below = (first >= 64) ? ~0ull : ((1ull << first) - 1);
        const int nm = __builtin_popcountll((bmatch >> (g * G)) & gmask & below);
        const uint32_t gcode = (uint32_t)wv_shfl((int)code, g * G + (first < G ? first : 0));
        if (walking) {
            if (first > 0) {
                if (!run) w.nent++;
                if (emit) run += first; else run = 1;
                w.len += first; w.idn += nm; px -= first; py -= first;
            }
            if (first < G && px > 0 && py > 0) {          // a jump at (px,py)
                const int src = (int)(gcode & 0x3FFFu);
                const bool up = (gcode >> 14) == 2u;
                int n;
                if (up) { n = px - src; px = src; py -= 1; }    // X run vs '-'  (:520-530)
                else    { n = py - src; py = src; px -= 1; }    // '-' vs Y run  (:531-543)
                if (n < 1 || (gcode >> 14) < 2u) { w.bad = true; walking = false; }
                if (emit && gl == 0 && !w.bad) {
                    if (run) path[w.nent - 1] = (IMSAME_MOVE_DIAG << 30) | (uint32_t)run;
                    path[w.nent] = ((up ? IMSAME_MOVE_UP : IMSAME_MOVE_LEFT) << 30) | (uint32_t)n;
                }
                w.nent++;
                run = 0;
                w.len += n; w.eg += n - 1; w.ig += 1;
            }
            walking = walking && px > 0 && py > 0;
            if (--guard < 0) { w.bad = true; walking = false; }
        }
    }
    if (emit && gl == 0 && run) path[w.nent - 1] = (IMSAME_MOVE_DIAG << 30) | (uint32_t)run;
    w.cx = px; w.cy = py;
    return w;
}

// One wave's share of a launch: pulls groups of GPW candidates from the work
// queue until it is empty.  wsm = this wave's LDS (nw_wave_lds bytes).
__device__ void nw_wave(const NwLaunch &P, uint8_t *wsm, const int lane, const uint32_t slot) {
    const int G = P.G, GPW = P.GPW;
    const int g = lane / G, gl = lane - g * G;
    const bool in_group = g < GPW;
    int *red = (int *)(wsm + GPW * P.xstride);                      // 64 x 4 ints
    uint32_t *tbw = P.tb + (uint64_t)slot * P.tb_wave_dw;
    const uint16_t *tb16 = (const uint16_t *)tbw;
    int *bnd = P.bnd + (uint64_t)slot * P.bnd_wave;
    const int ig = P.igap, eg = P.egap;

    for (;;) {
        uint32_t base = 0;
        if (lane == 0) base = wv_atomic_add(P.counter, (uint32_t)GPW);
        base = wv_first(base);
        if (base >= P.n_cand) break;
        const uint32_t c = base + g;
        const bool cvalid = in_group && c < P.n_cand;
        int xlen = 0, ylen = 0;
        uint64_t xo = 0, yo = 0;
        uint32_t sid = 0;
        if (cvalid) {
            const uint32_t rd = P.cand_read[c];
            sid = P.cand_sid[c];
            xo = P.db_start[sid]; xlen = (int)(P.db_start[sid + 1] - xo);
            yo = P.q_start[rd];   ylen = (int)(P.q_start[rd + 1] - yo);
        }
        uint8_t *X = wsm + (in_group ? g : 0) * P.xstride;
        if (cvalid)
            for (int k = gl; k < xlen; k += G) X[k] = P.db[xo + k];
        wv_lds_sync();

        int xmax = xlen, nstr = cvalid ? (ylen + NW_W - 1) / NW_W : 0;
        for (int o = 32; o > 0; o >>= 1) {
            xmax = max(xmax, wv_shfl_xor(xmax, o));
            nstr = max(nstr, wv_shfl_xor(nstr, o));
        }
        int bestR = INT_MIN, bestRj = 0, bestC = INT_MIN, bestCi = 0;
        const int lastj = ylen - 1;

        for (int st = 0; st < nstr; ++st) {
            const int j0 = st * NW_W + gl * NW_K;
            const bool lact = cvalid && j0 < ylen;
            const bool leadc0 = (gl == 0) && st == 0;
            const bool lead_seam = (gl == 0) && st > 0;
            const bool seam_out = (gl == G - 1) && (st + 1) * NW_W < ylen && cvalid;
            const bool owns_last = cvalid && lastj >= j0 && lastj < j0 + NW_K;
            const int s_last = lastj - j0;
            int Y[NW_K], cJ[NW_K], colc[NW_K], colcode[NW_K];
#pragma unroll
            for (int s = 0; s < NW_K; ++s) {
                const int j = j0 + s;
                Y[s] = (cvalid && j < ylen) ? (int)P.q[yo + j] : 0;
                cJ[s] = (j <= 1) ? -NW_BIG : ig + (j - 1) * eg;        // left needs j > 1 (:443)
                colc[s] = -eg * (j - 1);
                colcode[s] = 0xC000 | ((j - 1) & 0x3FFF);
            }
            // row 0 (alignmentFunctions.c:404-413): T[0][j] = s(X0,Yj), mc[j] = (T[0][j], row 0)
            const int x0 = cvalid ? (int)X[0] : 0;
            const int yprev = (cvalid && j0 > 0) ? (int)P.q[yo + j0 - 1] : 0;
            const int t0prev = (x0 == yprev) ? 4 : -4;
            int own[NW_K], own2[NW_K], mcS[NW_K], mcAdj[NW_K], mcCode[NW_K];
#pragma unroll
            for (int s = 0; s < NW_K; ++s) {
                own[s] = (x0 == Y[s]) ? 4 : -4;
                own2[s] = -NW_BIG;
            }
#pragma unroll
            for (int s = 0; s < NW_K; ++s) {
                mcS[s] = (s == 0) ? t0prev : own[s - 1];
                mcAdj[s] = mcS[s];
                mcCode[s] = 0x8000;
                if (j0 + s == 1) mcS[s] = NW_BIG;     // mc[0] is never updated (j > 1 test, :476)
            }
            int in1 = t0prev, in2 = -NW_BIG;
            int outT = own[NW_K - 1], outMS = 0, outMC = 0;
            const int tend = xmax - 1 + G;
            for (int t = 1; t < tend; ++t) {
                int sN = wv_shr1(outT), mS = wv_shr1(outMS), mC = wv_shr1(outMC);
                const int i = t - gl;
                const bool act = lact && i >= 1 && i < xlen;
                if (lead_seam && act) { sN = bnd[3 * i]; mS = bnd[3 * i + 1]; mC = bnd[3 * i + 2]; }
                if (act) {
                    const int xi = X[i];
                    const int cI = (i == 1) ? -NW_BIG : ig + (i - 1) * eg;   // up needs i > 1 (:449)
                    const int rowc2 = -eg * (i - 2);
                    const int code2 = 0x8000 | ((i - 2) & 0x3FFF);
                    int mfS = mS, mfCode = mC, mfAdj = mS - eg * (mC & 0x3FFF);
                    int cur[NW_K];
                    uint32_t code[NW_K];
#pragma unroll
                    for (int s = 0; s < NW_K; ++s) {
                        const int d0 = (s == 0) ? in1 : own[s - 1];     // T[i-1][j-1]
                        const int u2 = (s == 0) ? in2 : own2[s - 1];    // T[i-2][j-1]
                        const int tl = (s == 0) ? sN : cur[s - 1];      // T[i][j-1]
                        const bool m = xi == Y[s];
                        const int sc = m ? 4 : -4;
                        const int l0 = mfAdj + cJ[s];                   // left  - s  (:444)
                        const int u0 = mcAdj[s] + cI;                   // up    - s  (:450)
                        const int mx = max(l0, u0);
                        int v = max(d0, mx) + sc;
                        // diag if >= both, else up if up > left, else left (:457-472)
                        const uint32_t cd = (d0 >= mx) ? (uint32_t)m : (uint32_t)((u0 > l0) ? mcCode[s] : mfCode);
                        if (s == 0) v = leadc0 ? sc : v;                 // column 0 (:426)
                        cur[s] = v;
                        code[s] = cd;
                        // column max of column j-1 over rows <= i-2, strict > (:476-480)
                        if (u2 > mcS[s]) { mcS[s] = u2; mcAdj[s] = u2 + rowc2; mcCode[s] = code2; }
                        // row state for column j+1: tested on row i, taken from row i-1 (:434-438)
                        if (mfS <= tl) { mfS = d0; mfAdj = d0 + colc[s]; mfCode = colcode[s]; }
                        if (s == 0) mfS = leadc0 ? -NW_BIG : mfS;        // then mf = T[i-1][0]
                    }
                    uint32_t *dst = tbw + (((uint32_t)st * P.steps + t) * 64u + lane) * NW_KW;
                    dst[0] = code[0] | (code[1] << 16);
                    dst[1] = code[2] | (code[3] << 16);
                    dst[2] = code[4];
                    if (i == xlen - 1) {                                 // last row (:481)
#pragma unroll
                        for (int s = 0; s < NW_K; ++s) {
                            const int j = j0 + s;
                            if (j >= 1 && j < ylen && cur[s] >= bestR) { bestR = cur[s]; bestRj = j; }
                        }
                    } else if (owns_last) {                              // last column, rows < xlen-1
                        int v = cur[0];
#pragma unroll
                        for (int s = 1; s < NW_K; ++s) v = (s_last == s) ? cur[s] : v;
                        if (v >= bestC) { bestC = v; bestCi = i; }
                    }
                    in2 = in1; in1 = sN;
#pragma unroll
                    for (int s = 0; s < NW_K; ++s) { own2[s] = own[s]; own[s] = cur[s]; }
                    outT = cur[NW_K - 1]; outMS = mfS; outMC = mfCode;
                    if (seam_out) { bnd[3 * i] = outT; bnd[3 * i + 1] = mfS; bnd[3 * i + 2] = mfCode; }
                }
            }
            wv_mem_sync();
        }

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
        if (bR >= bC) { bscore = bR; bx = xlen - 1; by = bRj; }
        else          { bscore = bC; bx = bCi; by = ylen - 1; }
        wv_lds_sync();

        const int gg = in_group ? g : 0;
        WalkOut w = nw_walk(tb16, bx, by, cvalid, gg, gl, G, P.steps, nullptr, false);
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
            nw_walk(tb16, bx, by, ok, gg, gl, G, P.steps, ok ? P.paths + off : nullptr, true);
            if (ok) { poff = off; plen = (uint32_t)w.nent; }
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
        wv_lds_sync();
    }
}

// Launch shape for reads up to ymax and records up to xcap: short reads pack
// 64/G candidates per wave, long reads take a wave each over several strips;
// X staging is capped at 16 KB of LDS per wave.
struct NwShape { int G, GPW, nstr, xcap, xstride, steps; };
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

#ifndef IMSAME_WAVE_EMU
__global__ __launch_bounds__(256) void nw_kernel(NwLaunch P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    const uint32_t slot = blockIdx.x * (blockDim.x >> 6) + wib;
    nw_wave(P, smem + wib * nw_wave_lds(P.GPW, P.xstride), lane, slot);
}
#endif
