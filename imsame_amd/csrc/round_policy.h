// round_policy.h -- the decisions of the read scheduler's rounds, shared by
// the device library (imsame_dev.hip:align_one) and the CPU wave emulator
// (tests/emu/wave_emu.cpp:emu_align), so that a policy change is made once:
// the candidate lists' capacity, speculation widths, per-round hit budgets,
// scan group sizes and when round 1b runs.  Host code; included after
// seed_kernel.hip (SPEC_*, SEED_BUDGET1, seed_budget, seed_lanes).
//
// Reference: the reads' scan order and acceptance are computeAlignmentsByThread's
// (alignmentFunctions.c:43-208); none of these choices changes a result, only
// how the scan is cut into rounds (tests run every knob against the oracle).
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <algorithm>

struct RoundPolicy {
    uint32_t spec_weak = 1;          // candidates from a read's first weak candidate on (spec_after_first)
    uint32_t spec_later = SPEC_MAX;  // candidates per read in rounds >= 2
    bool spec_set = false;           // IMSAME_SPEC given: no SPEC_BIG widening for whole-wave groups
    uint64_t ccap = 0;               // entries of each candidate list
    uint32_t budget1 = SEED_BUDGET1; // round 1's hit budget per read; later rounds x grow
    uint32_t grow = 8;
    uint64_t l64_below = 8192;       // reads (over all lanes) below which a whole wave scans a read
    int nlanes = 1;                  // lanes of the call: the device scans nlanes x na reads at once
    bool r1b_on = true;              // round 1b (short reads only)
    bool split_on = true;            // split rounds (imsame_dev.hip:align_one; short reads only)
    uint32_t split_min = 16384;      // ... of at least this many active reads
    bool window = true;              // predicted traceback windows of the packed NW kernel
    bool weak_rows = false;          // ... predicted from weak hits too (IMSAME_NW_WEAK_ROWS)
    bool r1b_rows = false;           // ... for round 1b's candidates (IMSAME_NW_R1B_ROWS)

    // A lane's call of n reads whose longest is ycap (short reads: <= short_y).
    // Environment overrides (A/B runs, tests): IMSAME_SPEC_WEAK, IMSAME_CCAP_MULT,
    // IMSAME_SPEC, IMSAME_SEED_BUDGET, IMSAME_SEED_GROW, IMSAME_SEED_L64,
    // IMSAME_ROUND1B, IMSAME_NW_WINDOW.
    static RoundPolicy make(uint64_t n, uint32_t ycap, uint32_t short_y, int nlanes) {
        RoundPolicy r;
        r.nlanes = std::max(1, nlanes);
        const char *sw = getenv("IMSAME_SPEC_WEAK");
        r.spec_weak = (uint32_t)std::max(1, std::min(SPEC_MAX, sw ? atoi(sw) : SPEC_WEAK));
        // candidate lists: 2 per read (up to SPEC_MAX for small calls -- long
        // reads, few per call, fill launches by speculating); IMSAME_CCAP_MULT:
        // candidates per read the lists hold (round 1b's speculation width is
        // bounded by the room round 1 leaves)
        const char *cm = getenv("IMSAME_CCAP_MULT");
        const uint64_t cmult = cm ? (uint64_t)std::max(2, std::min(SPEC_BIG, atoi(cm))) : 2u;
        r.ccap = std::max<uint64_t>(n * std::max<uint64_t>(r.spec_weak > 1 ? r.spec_weak + 1 : 2, cmult),
                                    std::min<uint64_t>(n * SPEC_MAX, 1u << 20));
        // speculation: round 1 emits one candidate per read (most reads accept
        // it); later rounds up to SPEC_MAX, bounded by the lists
        const char *sp = getenv("IMSAME_SPEC");
        r.spec_set = sp != nullptr;
        r.spec_later = sp ? (uint32_t)std::max(1, std::min(SPEC_MAX, atoi(sp))) : (uint32_t)SPEC_MAX;
        const char *bu = getenv("IMSAME_SEED_BUDGET");
        // (2 x SEED_BUDGET1 for lanes of >= 200k reads -- C2 and C3's lanes:
        // C3 392.4 -> 383.8 ms, C2 106.2 -> 105.8-105.9 ms per step; a lane of
        // the 1/4 shard's 83k reads ran 29.8 ms against 28.6, profiles/r5zg/)
        r.budget1 = bu ? (uint32_t)std::max(0, atoi(bu)) : (n >= 200000 ? 2 * SEED_BUDGET1 : SEED_BUDGET1);
        // budget growth per round: 8x; a lane of < 100k reads (an 8-GPU shard
        // of C2) 64x, so its third round finishes the random reads' scans
        // instead of leaving a latency-bound fourth round of tiny launches (C2
        // shard 1/8: 23.4 -> 20.1 ms per step; no effect from 1/4 up,
        // profiles/r2u_*, r2v_*)
        const char *gr = getenv("IMSAME_SEED_GROW");
        r.grow = gr ? (uint32_t)std::max(2, atoi(gr)) : (n < 100000 ? 64u : 8u);
        // (C2 1/8 shard: 18.5 vs 19.2 ms per step, round 2's ~2k reads scan in
        // a third of the time; 32768 also takes round 1b's 17k: 18.9; C2
        // unchanged; profiles/r3l64/)
        const char *l64 = getenv("IMSAME_SEED_L64");
        r.l64_below = l64 ? strtoull(l64, nullptr, 10) : 8192;
        const char *rb = getenv("IMSAME_ROUND1B");
        r.r1b_on = !(rb && !atoi(rb)) && ycap <= short_y;
        const char *sr = getenv("IMSAME_SPLIT_ROUNDS"), *sm = getenv("IMSAME_SPLIT_MIN");
        r.split_on = !(sr && !atoi(sr)) && ycap <= short_y;
        if (sm) r.split_min = (uint32_t)std::max(2, atoi(sm));
        // (round 2 measured the windows 1-3 % slower -- the window steps spilled
        // at 4 waves per SIMD, round 1b off; at 3 waves per SIMD and with round
        // 1b they take C2's NW busy time from 113.4 to 107.4 ms, profiles/r4d/)
        const char *wi = getenv("IMSAME_NW_WINDOW");
        r.window = !(wi && !atoi(wi));
        const char *wr = getenv("IMSAME_NW_WEAK_ROWS"), *br = getenv("IMSAME_NW_R1B_ROWS");
        r.weak_rows = wr && atoi(wr);
        r.r1b_rows = br && atoi(br);
        return r;
    }
    // lanes per read of round `round`'s scan of na reads: from the reads the
    // device scans at once (this lane's times the call's lanes; C2, 8 lanes of
    // 125k: 4 lanes per read in round 1 instead of 16, whose extra windows a
    // true read never needs, +1.9 %, profiles/r2am_*), and a whole wave per
    // read where few reads scan (their remaining windows 64 at a time; those
    // groups may emit up to SPEC_BIG candidates).  IMSAME_SEED_L (round 1:
    // IMSAME_SEED_L1 if set) forces it.
    int pick_L(uint32_t round, uint32_t na) const {
        const char *le = getenv(round == 1 && getenv("IMSAME_SEED_L1") ? "IMSAME_SEED_L1" : "IMSAME_SEED_L");
        if (le) return atoi(le);
        const uint64_t all = (uint64_t)na * (uint64_t)nlanes;
        return all < l64_below ? 64 : seed_lanes((uint32_t)std::min<uint64_t>(all, 0xFFFFFFFFu));
    }
    // candidates per read of round `round` (nact reads scanning): the round's
    // candidates fit the lists (nact x spec <= ccap); whole-wave groups up to
    // SPEC_BIG
    uint32_t spec(uint32_t round, uint32_t nact) const {
        if (round == 1) return 1;
        const uint64_t room = ccap / std::max<uint32_t>(nact, 1);
        const uint64_t w = (!spec_set && pick_L(round, nact) >= 64) ? SPEC_BIG : spec_later;
        return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(w, room));
    }
    uint32_t budget(uint32_t round) const { return seed_budget(budget1, round, grow); }
    // Round 1b: round 1 paused reads without a candidate, no long-read
    // candidates, and the lists have room after round 1's n1
    bool r1b(uint32_t round, uint64_t n1, uint64_t n2, uint64_t paused) const {
        return round == 1 && r1b_on && paused > 0 && n2 == 0 && ccap > n1;
    }
    // ... its scan: weak-first speculation up to SPEC_MAX per read, SPEC_BIG
    // where whole-wave groups scan (their lists hold it), in the room left;
    // round 2's budget
    uint32_t r1b_spec_weak(uint64_t n1, uint32_t paused) const {
        const uint64_t w = pick_L(1, paused) >= 64 ? SPEC_BIG : SPEC_MAX;
        return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(w, (ccap - n1) / std::max<uint32_t>(paused, 1)));
    }
    uint32_t r1b_budget() const { return seed_budget(budget1, 2, grow); }
    // Split rounds: a round >= 2 of at least split_min active reads scans
    // them in two halves, each half's NW launch starting after its own scan
    bool split(uint32_t round, uint32_t nact) const {
        return round >= 2 && split_on && nact >= split_min;
    }
};
