// wave_emu.cpp -- TEST INFRASTRUCTURE: runs the device kernel source
// (imsame_amd/csrc/{nw,seed}_kernel.hip) on the CPU.  Each wave is 64 lanes
// on ONE host thread as user-space fibers (ucontext): a lane runs until its
// next cross-lane op, which hands over to the next lane, so DPP / ballot /
// shuffle are lock-step exchanges (wave_ops.h, IMSAME_WAVE_EMU) at the cost
// of 64 context switches.  Launches run several waves on host threads, each
// with its own arena slot, as the device does.  Sanitizer builds
// (scripts/sanitize.sh) use one host thread per lane and a barrier instead.
// The round orchestration below mirrors imsame_dev.hip:imsame_dev_align with
// host memory in place of HBM.  Built by tests/emu/Makefile into
// tests/emu/build/libwave_emu.so.
#define IMSAME_WAVE_EMU 1
#include <algorithm>
#include <atomic>
#include <functional>
#include <memory>
#include <thread>
#include <vector>
#include <stdio.h>
#include <string.h>
#include <math.h>
#if defined(__SANITIZE_ADDRESS__) || defined(__SANITIZE_THREAD__)
#define EMU_THREADS 1
#include <barrier>
#else
#include <ucontext.h>
#endif
#include "../../imsame_amd/csrc/wave_ops.h"

namespace wvemu {
thread_local Wave *t_wave;
thread_local int t_lane;
thread_local uint64_t *t_xch;
#ifdef EMU_THREADS
struct Wave {
    std::barrier<> bar{64};
    uint64_t xch[64];
};
void sync() { t_wave->bar.arrive_and_wait(); }
#else
struct Wave {
    ucontext_t ctx[64], caller;
    uint64_t xch[64];
    const std::function<void(int)> *f;
    std::unique_ptr<char[]> stacks;
};
constexpr size_t STACK = 1u << 20;
// every lane has arrived once the last one hands over to lane 0
void sync() {
    Wave *w = t_wave;
    const int me = t_lane, nx = (me + 1) & 63;
    t_lane = nx;
    swapcontext(&w->ctx[me], &w->ctx[nx]);
}
// a lane's body; when it ends, the next lane (waiting in its last sync) ends
// too, and the last one returns to the caller
static void fiber_entry() {
    Wave *w = t_wave;
    const int l = t_lane;
    (*w->f)(l);
    if (l < 63) { t_lane = l + 1; setcontext(&w->ctx[l + 1]); }
    setcontext(&w->caller);
}
#endif
}  // namespace wvemu

#include "../../include/imsame_dev.h"
#include "../../imsame_amd/csrc/tables.h"
#include "../../imsame_amd/csrc/nw_kernel.hip"
#include "../../imsame_amd/csrc/nw16_kernel.hip"
#include "../../imsame_amd/csrc/nwl_kernel.hip"
#include "../../imsame_amd/csrc/nwp_kernel.hip"
#include "../../imsame_amd/csrc/seed_kernel.hip"
#include "../../imsame_amd/csrc/round_policy.h"

static void run_wave(const std::function<void(int)> &f) {
#ifdef EMU_THREADS
    wvemu::Wave w;
    std::vector<std::thread> th;
    th.reserve(64);
    for (int l = 0; l < 64; ++l)
        th.emplace_back([&w, &f, l] {
            wvemu::t_wave = &w; wvemu::t_lane = l; wvemu::t_xch = w.xch;
            f(l);
        });
    for (auto &t : th) t.join();
#else
    auto w = std::make_unique<wvemu::Wave>();
    w->f = &f;
    w->stacks.reset(new char[64 * wvemu::STACK]);
    for (int l = 0; l < 64; ++l) {
        getcontext(&w->ctx[l]);
        w->ctx[l].uc_stack.ss_sp = w->stacks.get() + (size_t)l * wvemu::STACK;
        w->ctx[l].uc_stack.ss_size = wvemu::STACK;
        w->ctx[l].uc_link = nullptr;
        makecontext(&w->ctx[l], wvemu::fiber_entry, 0);
    }
    wvemu::t_wave = w.get(); wvemu::t_lane = 0; wvemu::t_xch = w->xch;
    swapcontext(&w->caller, &w->ctx[0]);
    wvemu::t_wave = nullptr;
#endif
}

// waves w = 0 .. nw-1 of one launch, each on a host thread of its own: f(lane, w)
static void run_waves(int nw, const std::function<void(int, int)> &f) {
    std::vector<std::thread> th;
    for (int w = 1; w < nw; ++w) th.emplace_back([&f, w] { run_wave([&f, w](int l) { f(l, w); }); });
    run_wave([&f](int l) { f(l, 0); });
    for (auto &t : th) t.join();
}
// host threads the launches use (each wave holds a 64 MB stack block)
static int emu_threads() {
    const char *e = getenv("IMSAME_EMU_THREADS");
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    return std::max(1, e ? atoi(e) : std::min(hw, 8));
}

// waves whose nw16 traceback band missed a path (NwLaunch::redo), since the last emu_redo_count()
static uint32_t g_redo;
extern "C" uint32_t emu_redo_count(void) { const uint32_t r = g_redo; g_redo = 0; return r; }
// reads the round-1b scan took over (imsame_dev.hip:align_one), since the last emu_r1b_count()
static uint32_t g_r1b;
extern "C" uint32_t emu_r1b_count(void) { const uint32_t r = g_r1b; g_r1b = 0; return r; }
// candidates walked inside their first-sweep traceback window (NwLaunch::win), since the last call
static uint32_t g_win;
extern "C" uint32_t emu_win_count(void) { const uint32_t r = g_win; g_win = 0; return r; }

// packed launches that ran the 19-column form (nw16_k19_ok), since the last emu_k19_count()
static uint32_t g_k19, g_k3;
extern "C" uint32_t emu_k19_count(void) { const uint32_t r = g_k19; g_k19 = 0; return r; }
extern "C" uint32_t emu_k3_count(void) { const uint32_t r = g_k3; g_k3 = 0; return r; }
// long-read launches that ran the packed kernel (nwp_fits), and its waves that
// fell back to the int32 path, since the last emu_nwp_count()
static uint32_t g_nwp, g_fbk;
// int16 wraps the emulated nwp_kernel met in live cells (nwp_kernel.hip:nwp_chk)
std::atomic<uint64_t> g_nwp_viol{0};
extern "C" uint64_t emu_nwp_range_violations(void) { return g_nwp_viol.exchange(0); }
// nwp_chk on wraps of each kind (two adds, a sign, a decrement) and on the same operations in range: 4
extern "C" uint32_t emu_nwp_chk_selftest(void) {
    const uint64_t before = g_nwp_viol.exchange(0);
    nwp_chk(1u, 0, 0x0000FFF0u, 0x00000020u);      // low half: 0xFFF0 + 32 > 0xFFFF
    nwp_chk(2u, 0, 0xFFF0FFF0u, 0x0020FFE0u);      // high half: wraps; low: 0xFFF0 - 32 (not checked)
    nwp_chk(1u, 1, 0x00009000u, 0x00001000u);      // 0x8000 apart: the sign wraps
    nwp_chk(3u, 1, 0x80008000u, 0x00010001u);      // 0x7FFF apart: in range
    nwp_chk(2u, 2, 0x00010005u, 0x00020002u);      // high half 1 < 2: underflow
    nwp_chk(3u, 2, 0x00020002u, 0x00020002u);      // equal: in range
    const uint64_t n = g_nwp_viol.exchange(before);
    return (uint32_t)n;
}
extern "C" uint32_t emu_nwp_count(uint32_t *fallbacks) {
    const uint32_t r = g_nwp;
    if (fallbacks) *fallbacks = g_fbk;
    g_nwp = g_fbk = 0;
    return r;
}

static int run_nw(const uint8_t *db, const uint64_t *dbs, const uint8_t *q, const uint64_t *qs,
                  const uint32_t *cread, const uint32_t *csid, uint32_t n, const imsame_params *p, uint32_t ymax,
                  uint32_t xmax, const std::vector<uint32_t> &ml, const std::vector<uint32_t> &mi,
                  imsame_read_result *out, uint32_t *paths, uint32_t pcap, uint32_t *pused, uint32_t *flags,
                  const int32_t *crow = nullptr) {
    // same kernel choice as imsame_dev.hip:plan_nw
    const bool pk = !(p->flags & IMSAME_FLAG_NW32) && nw16_fits(p->igap, p->egap, xmax, ymax);
    const char *op = getenv("IMSAME_NW_ONEPASS");
    const bool two = pk && !(p->flags & IMSAME_FLAG_NW16_ONEPASS) && !(op && atoi(op));
    const char *le = getenv("IMSAME_NWL");
    const bool lng = !pk && !(p->flags & IMSAME_FLAG_NW32) && !(le && !atoi(le)) && nwl_fits(p->igap, p->egap, ymax);
    const char *pe = getenv("IMSAME_NWP");
    const bool lp = lng && !(pe && !atoi(pe)) && nwp_fits(p->igap, p->egap, xmax, ymax);
    // columns per lane of the packed kernel: imsame_dev.hip:nw16_k picks by the
    // chip's fill; here IMSAME_NW_K=5 selects the latency-bound form
    const char *ke = getenv("IMSAME_NW_K");
    uint32_t yuni = n ? (uint32_t)(qs[cread[0] + 1] - qs[cread[0]]) : 0;    // one read length? (nw16_k19_ok)
    for (uint32_t k = 0; k < n; ++k) if (qs[cread[k] + 1] - qs[cread[k]] != yuni) yuni = 0;
    int K = (ke && atoi(ke) == NW16_K5) ? NW16_K5
          : (pk && nw16_k19_ok(yuni, ymax, xmax, p)) ? NW16_K19 : NW16_K;
    // IMSAME_NW_K=3: the latency form where it applies (imsame_dev.hip:plan_nw)
    if (ke && atoi(ke) == NW16_K3)
        K = (ymax <= NW16_K3_YMAX && nw16_fits(p->igap, p->egap, xmax, ymax, NW16_K3)) ? NW16_K3 : NW16_K5;
    const NwShape sh = pk ? nw16_shape(ymax, xmax, K) : lp ? nwp_shape(ymax, xmax) : lng ? nwl_shape(ymax, xmax)
                     : nw_shape(ymax, xmax);
    // waves of the launch (one arena slot each), as many as it has tasks
    const uint32_t cpw = (pk || lp) ? 2u * (uint32_t)sh.GPW : (uint32_t)sh.GPW;
    const int nwv = (int)std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)emu_threads(), (n + cpw - 1) / cpw));
    const size_t tb_slot = (pk ? nw16_tb_words(sh) : lp ? nwp_tb_words(sh, ymax) : lng ? nwl_tb_words(sh, ymax)
                            : nw_tb_words(sh)) + 64;
    const size_t ck_slot = two ? nw16_ck_words(sh) : lp ? nwp_ck_words(sh, ymax) : lng ? nwl_ck_words(sh) : 1;
    std::vector<uint32_t> tb(tb_slot * nwv, 0xABABABABu);
    std::vector<uint32_t> ck(ck_slot * nwv, 0xCDCDCDCDu);
    const char *be = getenv("IMSAME_NW_BAND");
    // seam scratch poisoned like fresh device memory: a read before its write shows
    const size_t bnd_slot = (lp ? nwp_seam_words(sh, ymax) : lng ? nwl_seam_words(sh) : (size_t)3 * sh.xcap) + 64;
    std::vector<int32_t> bnd(bnd_slot * nwv, 0x70000000);
    const size_t lds_slot = (pk ? nw16_wave_lds(sh.GPW, sh.xstride)
                              : lng ? nwl_wave_lds(sh.xstride) : nw_wave_lds(sh.GPW, sh.xstride)) + 64;
    std::vector<uint8_t> lds(lds_slot * nwv, 0xA5);
    uint32_t counter = 0;
    NwLaunch P;
    memset(&P, 0, sizeof P);
    P.db = db; P.db_start = dbs; P.q = q; P.q_start = qs;
    P.cand_read = cread; P.cand_sid = csid; P.n_cand = n;
    P.igap = (int32_t)p->igap; P.egap = (int32_t)p->egap;
    P.G = sh.G; P.GPW = sh.GPW; P.xcap = sh.xcap; P.xstride = sh.xstride; P.steps = sh.steps;
    P.tb = tb.data(); P.tb_wave_dw = tb_slot;
    P.bnd = bnd.data(); P.bnd_wave = bnd_slot;
    P.minlen = ml.data(); P.n_minlen = ymax + 1;
    P.minident = mi.data(); P.n_minident = xmax + ymax + 2;
    P.counter = &counter; P.out = out;
    P.paths = paths; P.paths_cap = pcap; P.paths_used = pused; P.want_paths = p->want_paths;
    P.flags = flags;
    P.ck = ck.data(); P.ck_wave_dw = ck_slot;
    P.band_w = be ? std::max(0, atoi(be)) : 200;        // imsame_dev.hip:nw16_band_rows
    if (lng) {                                            // imsame_dev.hip:plan_nw
        const char *nb = getenv("IMSAME_NWL_BAND");
        P.band_w = nb ? std::max(1, std::min(NWL_BAND, atoi(nb))) : NWL_BAND_DEF;
    }
    P.redo = &g_redo;
    if (lp) {                                             // imsame_dev.hip:launch_nw
        P.rlim = (int32_t)nwp_rlim(p->igap, p->egap, (uint64_t)sh.xcap, ymax);
        const char *ns = getenv("IMSAME_NWP_S");
        P.nwp_s = ns ? atoi(ns) : 0;
        P.fbk = &g_fbk;
    }
    // queue order by predicted row, as imsame_dev.hip:launch_nw (row_bucket:
    // 8-row buckets, unpredicted first; stable here, any order is correct)
    std::vector<uint32_t> perm;
    if (crow && two && n >= 64) {
        const uint32_t nb = ((uint32_t)sh.xcap + 512) / 8 + 2;
        auto bucket = [&](int32_t r) -> uint32_t {
            if (r == INT32_MIN) return 0;
            const int64_t b = (((int64_t)r + 256) >> 3) + 1;
            return (uint32_t)(b < 1 ? 1 : b > (int64_t)nb - 1 ? (int64_t)nb - 1 : b);
        };
        std::vector<uint32_t> cur(nb + 1, 0);
        for (uint32_t k = 0; k < n; ++k) cur[bucket(crow[k]) + 1]++;
        for (uint32_t b = 0; b < nb; ++b) cur[b + 1] += cur[b];
        perm.resize(n);
        for (uint32_t k = 0; k < n; ++k) perm[cur[bucket(crow[k])]++] = k;
        P.perm = perm.data(); P.cand_row = crow;
        P.win_up = NW16_WIN_UP; P.win_down = NW16_WIN_DOWN;
        const char *wb = getenv("IMSAME_NW_WIN_BOTTOM");
        P.win_bottom = wb ? atoi(wb) : NW16_WIN_BOTTOM;
    }
    P.win = &g_win;
    bool ymult = true;        // every read length a multiple of NW16_K (imsame_dev.hip: q_len_mult)
    for (uint32_t k = 0; k < n; ++k) ymult = ymult && (qs[cread[k] + 1] - qs[cread[k]]) % NW16_K == 0;
    if (lp) {
        ++g_nwp;
        run_waves(nwv, [&](int lane, int w) { nwp_wave(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
    }
    else if (lng)         run_waves(nwv, [&](int lane, int w) { nwl_wave(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
    else if (pk && K == NW16_K19) {
        ++g_k19;
        if (two) run_waves(nwv, [&](int lane, int w) { nw16_wave<NW16_K19, true, true, NW16_K19_OFF>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
        else     run_waves(nwv, [&](int lane, int w) { nw16_wave<NW16_K19, true, false, NW16_K19_OFF>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
    }
    else if (pk && K == NW16_K3) {
        ++g_k3;
        bool m3 = true;       // every read length a multiple of 3 (imsame_dev.hip:plan_nw's LAST for K = 3)
        for (uint32_t k = 0; k < n; ++k) m3 = m3 && (qs[cread[k] + 1] - qs[cread[k]]) == ymax && ymax % NW16_K3 == 0;
        if (two && m3)        run_waves(nwv, [&](int lane, int w) { nw16_wave<NW16_K3, true, true>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
        else if (two)         run_waves(nwv, [&](int lane, int w) { nw16_wave<NW16_K3, false, true>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
        else if (m3)          run_waves(nwv, [&](int lane, int w) { nw16_wave<NW16_K3, true, false>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
        else                  run_waves(nwv, [&](int lane, int w) { nw16_wave<NW16_K3, false, false>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
    }
    else if (pk && K == NW16_K5) {
        if (two && ymult)     run_waves(nwv, [&](int lane, int w) { nw16_wave<NW16_K5, true, true>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
        else if (two)         run_waves(nwv, [&](int lane, int w) { nw16_wave<NW16_K5, false, true>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
        else if (pk && ymult) run_waves(nwv, [&](int lane, int w) { nw16_wave<NW16_K5, true, false>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
        else if (pk)          run_waves(nwv, [&](int lane, int w) { nw16_wave<NW16_K5, false, false>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
    }
    else if (two && ymult) run_waves(nwv, [&](int lane, int w) { nw16_wave<NW16_K, true, true>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
    else if (two)         run_waves(nwv, [&](int lane, int w) { nw16_wave<NW16_K, false, true>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
    else if (pk && ymult) run_waves(nwv, [&](int lane, int w) { nw16_wave<NW16_K, true, false>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
    else if (pk)          run_waves(nwv, [&](int lane, int w) { nw16_wave<NW16_K, false, false>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
    else if (sh.nstr > 1) run_waves(nwv, [&](int lane, int w) { nw_wave<true>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
    else             run_waves(nwv, [&](int lane, int w) { nw_wave<false>(P, lds.data() + w * lds_slot, lane, (uint32_t)w); });
    if (const char *dump = getenv("IMSAME_EMU_DUMP_SEAM")) {       // debugging: the seam scratch as left
        if (FILE *f = fopen(dump, "wb")) { fwrite(bnd.data(), 4, bnd.size(), f); fclose(f); }
    }
    return 0;
}

extern "C" int emu_nw_pairs(const uint8_t *xs, const uint64_t *x_start, const uint8_t *ys, const uint64_t *y_start,
                            uint64_t npairs, const imsame_params *p, imsame_read_result *res, uint32_t *paths,
                            uint64_t paths_cap, uint64_t *paths_used, uint32_t *flags_out) {
    uint32_t xmax = 0, ymax = 0;
    for (uint64_t k = 0; k < npairs; ++k) {
        xmax = std::max<uint32_t>(xmax, (uint32_t)(x_start[k + 1] - x_start[k]));
        ymax = std::max<uint32_t>(ymax, (uint32_t)(y_start[k + 1] - y_start[k]));
    }
    if (!imsame_gaps_in_range(p->igap, p->egap, xmax, ymax)) return IMSAME_E_RANGE;
    std::vector<uint64_t> mr;
    std::vector<uint32_t> ml, mi, idx(npairs);
    imsame_build_tables(p, 1, ymax, xmax, mr, ml, mi);
    for (uint64_t k = 0; k < npairs; ++k) idx[k] = (uint32_t)k;
    uint32_t pused = 0, flags = 0;
    run_nw(xs, x_start, ys, y_start, idx.data(), idx.data(), (uint32_t)npairs, p, ymax, xmax, ml, mi, res, paths,
           (uint32_t)paths_cap, &pused, &flags);
    if (paths_used) *paths_used = pused;
    if (flags_out) *flags_out = flags;
    return (flags & 1) ? IMSAME_E_PATHS : 0;
}

// host CSR with the device index's semantics (imsame_dev.hip: kmer_code_kernel,
// kmer_scatter, segsort): buckets in descending pos
static void build_csr(const uint8_t *db, uint64_t L, const uint64_t *dbs, uint64_t n_db, const uint8_t *brk_in,
                      std::vector<uint64_t> &off, std::vector<uint2> &ent, bool abs) {
    std::vector<uint32_t> brk(L / 32 + 2, 0);
    if (brk_in) for (uint64_t b = 0; b < (L + 7) / 8; ++b) brk[b / 4] |= (uint32_t)brk_in[b] << (8 * (b % 4));
    for (uint64_t s = 0; s < n_db; ++s) if (dbs[s] < L) brk[dbs[s] >> 5] |= 1u << (dbs[s] & 31);
    std::vector<uint32_t> code(L, 0xFFFFFFFFu);
    off.assign(NBUCKETS + 1, 0);
    for (uint64_t p = IMSAME_FIXED_K - 1; p < L; ++p) {
        const uint64_t b0 = p - (IMSAME_FIXED_K - 2);
        const uint64_t win = ((uint64_t)brk[b0 >> 5] | ((uint64_t)brk[(b0 >> 5) + 1] << 32)) >> (b0 & 31);
        if (win & ((1u << (IMSAME_FIXED_K - 1)) - 1)) continue;
        uint32_t c = 0;
        for (int k = IMSAME_FIXED_K - 1; k >= 0; --k) c = (c << 2) | base2(db[p - k]);
        code[p] = c;
        off[c + 1]++;
    }
    for (uint32_t b = 0; b < NBUCKETS; ++b) off[b + 1] += off[b];
    ent.assign(off[NBUCKETS] + 1, uint2{0, 0});
    std::vector<uint64_t> fill(off.begin(), off.end() - 1);
    for (uint64_t p = L; p-- > 0;) {          // descending positions
        if (code[p] == 0xFFFFFFFFu) continue;
        uint64_t lo = 0, hi = n_db;
        while (hi - lo > 1) { uint64_t m = (lo + hi) / 2; if (dbs[m] <= p) lo = m; else hi = m; }
        ent[fill[code[p]]++] = uint2{(uint32_t)(p + 1 - (abs ? 0 : dbs[lo])), (uint32_t)lo};
    }
}

extern "C" int emu_align(const uint8_t *db, uint64_t db_len, const uint64_t *db_start, uint64_t n_db,
                         const uint8_t *db_brk, const uint8_t *q, uint64_t q_len, const uint64_t *q_start,
                         uint64_t n_q, uint64_t read_from, uint64_t read_to, uint64_t T, const imsame_params *p,
                         imsame_read_result *res, uint32_t *paths, uint64_t paths_cap, uint64_t *paths_used,
                         imsame_stats *stats) {
    std::vector<uint64_t> dbs(db_start, db_start + n_db), qs(q_start, q_start + n_q);
    dbs.push_back(db_len); qs.push_back(q_len);
    // aligned copies with the 64-byte tail padding the device buffers carry (chunked loads)
    std::vector<uint32_t> dbpad(db_len / 4 + 17, 0), qpad(q_len / 4 + 17, 0);
    if (db_len) memcpy(dbpad.data(), db, db_len);
    db = (const uint8_t *)dbpad.data();
    // The query as imsame_dev_set_query_range uploads a shard: only reads
    // [read_from, read_to) (their starts, bases and QPAD bases before them)
    // hold data; every other byte / start is POISON, so a kernel that used
    // anything outside the shard would diverge from the oracle.
    const uint64_t b0 = qs[read_from], b1 = qs[read_to], qbase = b0 > 64 ? b0 - 64 : 0;
    memset(qpad.data(), 0xEE, qpad.size() * 4);
    if (b1 > qbase) memcpy((uint8_t *)qpad.data() + qbase, q + qbase, b1 - qbase);
    memset((uint8_t *)qpad.data() + b1, 0, std::min<uint64_t>(64, qpad.size() * 4 - b1));
    q = (const uint8_t *)qpad.data();
    // the packed bases (imsame_dev.hip:pack2_kernel): the whole database, and
    // the query's words over [qbase, b1 + 64) as the upload packs them; other
    // words POISON
    std::vector<uint32_t> dbw(db_len / 16 + 4), qw(q_len / 16 + 8, 0xEEEEEEEEu);
    for (uint64_t w = 0; w < dbw.size(); ++w) dbw[w] = pk_word(db, (int64_t)w, 0, (int64_t)db_len);
    for (uint64_t w = qbase >> 4; w < std::min<uint64_t>(qw.size(), (b1 + 64) / 16 + 2); ++w)
        qw[w] = pk_word(q, (int64_t)w, (int64_t)qbase, (int64_t)std::min<uint64_t>(b1 + 64, qpad.size() * 4));
    std::vector<uint64_t> qsv(qs.size(), 0xDEADBEEFDEADBEEFull);
    for (uint64_t r = read_from; r <= read_to; ++r) qsv[r] = qs[r];
    uint64_t qlo_first = read_from;
    while (qlo_first > 0 && qs[qlo_first - 1] == qs[read_from]) --qlo_first;
    // the CSR of the last database is kept (tests align many shards against one)
    static std::vector<uint8_t> key;
    static std::vector<uint64_t> off;
    static std::vector<uint2> ent;
    std::vector<uint8_t> k2(db, db + db_len);
    k2.insert(k2.end(), (const uint8_t *)dbs.data(), (const uint8_t *)(dbs.data() + dbs.size()));
    if (db_brk) k2.insert(k2.end(), db_brk, db_brk + (db_len + 7) / 8);
    k2.push_back(db_brk ? 1 : 0);
    // the device's entry form (imsame_dev.hip:ent_abs_for)
    const char *er = getenv("IMSAME_ENT_REL");
    const bool ent_abs = !(er && atoi(er)) && db_len < 0xFFFFFFFFull;
    k2.push_back(ent_abs ? 1 : 0);
    if (k2 != key || off.empty()) {
        build_csr(db, db_len, dbs.data(), n_db, db_brk, off, ent, ent_abs);
        key.swap(k2);
    }
    uint32_t max_rec = 0, ymax = 0;
    for (uint64_t s = 0; s < n_db; ++s) max_rec = std::max<uint32_t>(max_rec, (uint32_t)(dbs[s + 1] - dbs[s]));
    for (uint64_t r = read_from; r < read_to; ++r) ymax = std::max<uint32_t>(ymax, (uint32_t)(qs[r + 1] - qs[r]));
    const uint32_t xcap = (uint32_t)std::min<uint64_t>(max_rec, p->max_read_size);
    const uint32_t ycap = (uint32_t)std::min<uint64_t>(ymax, p->max_read_size);
    if (!imsame_gaps_in_range(p->igap, p->egap, xcap, ycap)) return IMSAME_E_RANGE;
    std::vector<uint64_t> mr;
    std::vector<uint32_t> ml, mi;
    imsame_build_tables(p, db_len, ymax, xcap, mr, ml, mi);
    const uint32_t n = (uint32_t)(read_to - read_from);
    std::vector<uint64_t> cur_p(n);
    // the rounds' policy: the device's own (round_policy.h, imsame_dev.hip:align_one), one lane
    const uint32_t short_y = std::min<uint32_t>(ycap, NW_W / 2);
    const RoundPolicy RP = RoundPolicy::make(n, ycap, short_y, 1);
    const size_t ccap = RP.ccap;
    std::vector<uint32_t> cur_h(n), memo((size_t)n * MEMO), act(n), nxt(n), act2(n), cr(ccap), cs(ccap), cr2(ccap), cs2(ccap);
    std::vector<uint32_t> cbase(n), ccnt(n), perr(n);
    std::vector<int32_t> crow(ccap);
    int32_t *crowp = RP.window ? crow.data() : nullptr;
    std::vector<uint8_t> nmemo(n), rstat(n);
    std::vector<imsame_read_result> o1(ccap), o2(ccap);
    // per-candidate results poisoned like reused device buffers: a candidate the
    // NW kernels leave unwritten shows
    memset(o1.data(), 0xEE, o1.size() * sizeof(imsame_read_result));
    memset(o2.data(), 0xEE, o2.size() * sizeof(imsame_read_result));
    InitLaunch I = {qsv.data(), read_from, n, res, cur_p.data(), cur_h.data(), nmemo.data(), rstat.data(), act.data()};
    for (uint32_t k = 0; k < n; ++k) init_one(I, k);
    uint32_t nc[3] = {0, 0, 0}, pused = 0, flags = 0;
    unsigned long long err = ~0ull, nhits = 0, cells = 0, nacc = 0, swin = 0, sent = 0, sch = 0;
    uint32_t nact = n;
    imsame_stats st;
    memset(&st, 0, sizeof st);
    while (nact) {
        st.rounds++;
        nc[0] = nc[1] = nc[2] = 0;
        SeedLaunch S;
        S.db = db; S.db_start = dbs.data(); S.n_db = n_db; S.db_len = db_len;
        S.q = q; S.q_start = qsv.data(); S.n_q = n_q; S.q_len = q_len;
        S.dbw = dbw.data(); S.qw = qw.data();
        S.qs_lo = read_from; S.qs_lo_first = qlo_first;
        S.off = off.data(); S.ent = ent.data(); S.ent_abs = ent_abs; S.wcap = nullptr; S.wstart = nullptr;
        S.active = act.data(); S.n_active = nact;
        S.read_from = read_from; S.T = T ? T : 1;
        S.rpt = (uint64_t)floorl((long double)n_q / (long double)S.T);
        S.cur_p = cur_p.data(); S.cur_h = cur_h.data(); S.memo = memo.data(); S.nmemo = nmemo.data();
        S.rstat = rstat.data();
        S.minraw = mr.data(); S.n_minraw = ymax + 1;
        S.minlen = ml.data(); S.n_minlen = ymax + 1;
        S.minident = mi.data(); S.n_minident = xcap + ymax + 2;
        S.max_rs = p->max_read_size; S.short_ylen = short_y; S.max_rec = max_rec;
        const uint32_t rnd = (uint32_t)st.rounds;
        S.spec = RP.spec(rnd, nact);
        S.spec_weak = RP.spec_weak;
        S.budget = RP.budget(rnd);
        S.next = nxt.data(); S.nnext = &nc[2];
        S.cbase = cbase.data(); S.ccnt = ccnt.data(); S.perr = perr.data();
        S.cread = cr.data(); S.csid = cs.data(); S.ncand = &nc[0]; S.crow = crowp; S.weak_rows = RP.weak_rows;
        S.cread2 = cr2.data(); S.csid2 = cs2.data(); S.ncand2 = &nc[1];
        S.err = &err; S.nhits = &nhits;
        auto run_seed = [&](const SeedLaunch &SL, uint32_t na) {
            const int L = RP.pick_L(rnd, na);
            if (L <= 1) {
                for (uint32_t i = 0; i < na; ++i) {
                    SeedTally tl;
                    if (SL.ent_abs) seed_one<true>(SL, i, tl, g_ung_tab.v); else seed_one<false>(SL, i, tl, g_ung_tab.v);
                    nhits += tl.hits; swin += tl.wins; sent += tl.ents; sch += tl.chunks;
                }
            } else {                   // seed_group_kernel: 64-lane waves, several host threads
                const uint64_t nwaves = ((uint64_t)na * L + 63) / 64;
                const int nt = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)emu_threads(), nwaves));
                std::vector<uint2> lds((size_t)nt * 64 * SPEC_BIG);
                std::vector<uint32_t> gms((size_t)nt * 64 * MEMO);
                std::atomic<unsigned long long> wh{0}, ww{0}, we{0}, wc{0};
                std::atomic<uint64_t> next_wave{0};
                std::vector<std::thread> th;
                auto worker = [&](int t) {
                    for (uint64_t wv; (wv = next_wave++) < nwaves;) {
                        const uint64_t w0 = wv * 64;
                        uint2 *ld = lds.data() + (size_t)t * 64 * SPEC_BIG;
                        uint32_t *gmw = gms.data() + (size_t)t * 64 * MEMO;
                        run_wave([&](int lane) {
                            SeedTally h;
                            const uint32_t gidx = (uint32_t)((w0 + lane) / L);
                            if (L == 64) SL.ent_abs ? seed_group<64, SPEC_BIG, true>(SL, gidx, lane, lane, ld + lane * SPEC_BIG, h, g_ung_tab.v, gmw + (lane / L) * MEMO)
                                         : seed_group<64, SPEC_BIG, false>(SL, gidx, lane, lane, ld + lane * SPEC_BIG, h, g_ung_tab.v, gmw + (lane / L) * MEMO);
                            else if (L >= 16) SL.ent_abs ? seed_group<16, SPEC_MAX, true>(SL, gidx, lane % 16, lane, ld + lane * SPEC_MAX, h, g_ung_tab.v, gmw + (lane / L) * MEMO)
                                         : seed_group<16, SPEC_MAX, false>(SL, gidx, lane % 16, lane, ld + lane * SPEC_MAX, h, g_ung_tab.v, gmw + (lane / L) * MEMO);
                            else if (L >= 4) SL.ent_abs ? seed_group<4, SPEC_MAX, true>(SL, gidx, lane % 4, lane, ld + lane * SPEC_MAX, h, g_ung_tab.v, gmw + (lane / L) * MEMO)
                                         : seed_group<4, SPEC_MAX, false>(SL, gidx, lane % 4, lane, ld + lane * SPEC_MAX, h, g_ung_tab.v, gmw + (lane / L) * MEMO);
                            else         SL.ent_abs ? seed_group<2, SPEC_MAX, true>(SL, gidx, lane % 2, lane, ld + lane * SPEC_MAX, h, g_ung_tab.v, gmw + (lane / L) * MEMO)
                                         : seed_group<2, SPEC_MAX, false>(SL, gidx, lane % 2, lane, ld + lane * SPEC_MAX, h, g_ung_tab.v, gmw + (lane / L) * MEMO);
                            wh += h.hits; ww += h.wins; we += h.ents; wc += h.chunks;
                        });
                    }
                };
                for (int t = 1; t < nt; ++t) th.emplace_back(worker, t);
                worker(0);
                for (auto &x : th) x.join();
                nhits += wh; swin += ww; sent += we; sch += wc;
            }
        };
        auto nw_upd = [&](uint32_t *r, uint32_t *s_, uint32_t nc_, imsame_read_result *o, uint32_t y, const int32_t *row,
                          uint32_t *next, uint32_t *nnext) {
            run_nw(db, dbs.data(), q, qsv.data(), r, s_, nc_, p, y, xcap, ml, mi, o, paths,
                   (uint32_t)paths_cap, &pused, &flags, row);
            st.n_nw += nc_;
            UpdLaunch U = {r, s_, nc_, o, read_from, res, rstat.data(), memo.data(), nmemo.data(),
                           cbase.data(), ccnt.data(), perr.data(), cur_p.data(), next, nnext, &cells, &nacc, &err,
                           dbs.data()};
            for (uint32_t k = 0; k < nc_; ++k) {
                uint64_t ce = 0, ac = 0, wa = 0;
                update_one(U, k, ce, ac, wa);
                cells += ce; nacc += ac; st.nw_spec_waste += wa;
            }
        };
        run_seed(S, nact);
        if (nc[0] + nc[1] + nc[2] == 0) break;
        // round 1b (imsame_dev.hip:align_one): the reads round 1 paused scan on
        // (weak-first speculation, round 2's budget) before round 1's NW results
        if (RP.r1b(rnd, nc[0], nc[1], nc[2])) {
            const uint32_t n1 = nc[0], npz = nc[2];
            uint32_t nb[3] = {0, 0, 0};
            SeedLaunch Sb = S;
            Sb.active = nxt.data(); Sb.n_active = npz;
            Sb.spec = 1;
            Sb.spec_weak = RP.r1b_spec_weak(n1, npz);
            Sb.budget = RP.r1b_budget();
            Sb.next = act2.data(); Sb.nnext = &nb[2];
            Sb.cread = cr.data() + n1; Sb.csid = cs.data() + n1; Sb.ncand = &nb[0];
            Sb.crow = crowp && RP.r1b_rows ? crowp + n1 : nullptr;
            Sb.ncand2 = &nb[1];
            run_seed(Sb, npz);
            if (nb[1]) return IMSAME_E_STATE;
            if (n1) nw_upd(cr.data(), cs.data(), n1, o1.data(), short_y, crowp, act2.data(), &nb[2]);
            if (nb[0]) nw_upd(cr.data() + n1, cs.data() + n1, nb[0], o1.data() + n1, short_y, Sb.crow, act2.data(), &nb[2]);
            g_r1b += npz;
            if (getenv("IMSAME_DEBUG_ROUNDS"))
                fprintf(stderr, "[emu round 1b] paused=%u cand=%u+%u next=%u\n", npz, n1, nb[0], nb[2]);
            nact = nb[2];
            std::swap(act, act2);
            continue;
        }
        struct { uint32_t n; uint32_t *r, *s; imsame_read_result *o; uint32_t y; const int32_t *row; } cls[2] = {
            {nc[0], cr.data(), cs.data(), o1.data(), short_y, crowp}, {nc[1], cr2.data(), cs2.data(), o2.data(), ycap, nullptr}};
        for (auto &c : cls)
            if (c.n) nw_upd(c.r, c.s, c.n, c.o, c.y, c.row, nxt.data(), &nc[2]);
        nact = nc[2];
        std::swap(act, nxt);
    }
    st.n_reads = n; st.n_hits = nhits; st.nw_cells = cells; st.n_accepted = nacc;
    st.seed_windows = swin; st.seed_entries = sent; st.seed_ext_chunks = sch;
    st.err_read = ~0ull;
    int ret = 0;
    if (err != ~0ull) { st.err_read = err >> 32; st.err_dbseq = err & 0xFFFFFFFFull; ret = IMSAME_E_READ_TOO_LONG; }
    if (paths_used) *paths_used = pused;
    if ((flags & 1) && !ret) ret = IMSAME_E_PATHS;
    if (stats) *stats = st;
    return ret;
}

// seed_kernel.hip:ungapped_raw for one hit (pd0 = DB position after the
// seed, pq0 = query position after it), bounds as seed_one derives them
extern "C" uint64_t emu_ungapped(const uint8_t *db, uint64_t db_len, const uint64_t *db_start, uint64_t n_db,
                                 const uint8_t *q, uint64_t q_len, const uint64_t *q_start, uint64_t n_q,
                                 uint64_t pd0, uint64_t pq0, uint64_t read, uint64_t sid) {
    std::vector<uint32_t> dbw(db_len / 16 + 4), qw(q_len / 16 + 4);
    for (uint64_t w = 0; w < dbw.size(); ++w) dbw[w] = pk_word(db, (int64_t)w, 0, (int64_t)db_len);
    for (uint64_t w = 0; w < qw.size(); ++w) qw[w] = pk_word(q, (int64_t)w, 0, (int64_t)q_len);
    const int64_t xs = (int64_t)db_start[sid];
    const int64_t xe = (sid == n_db - 1) ? (int64_t)db_len : (int64_t)db_start[sid + 1] - 1;
    const int64_t ys = (int64_t)q_start[read];
    const int64_t ye = (read == n_q - 1) ? (int64_t)q_len : (int64_t)q_start[read + 1] - 1;
    return ungapped_raw(g_ung_tab.v, dbw.data(), qw.data(), (int64_t)pd0, (int64_t)pq0,
                        xs, xe, ys, ye, (int64_t)db_len, (int64_t)q_len);
}

// table entry points for tests/test_host.py
extern "C" uint64_t emu_minraw(uint64_t ylen, uint64_t Ldb, const imsame_params *p) {
    return imsame_minraw(ylen, Ldb, p->min_e);
}
extern "C" uint32_t emu_minnum(uint64_t den, uint64_t cap, const imsame_params *p, int identity) {
    return imsame_minnum(den, identity ? p->min_identity : p->min_coverage, cap);
}
