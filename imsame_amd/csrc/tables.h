// tables.h -- host-side exact integer thresholds for the device decisions.
//
// The reference decides with x87 long double arithmetic:
//   e-value   (long double)0.333 * ylen * L_db * expl(-0.275 * raw) < min_e
//                                                alignmentFunctions.c:384, :139
//   coverage  (long double)length / ylen      >= min_coverage    :163
//   identity  (long double)identities / length >= min_identity   :163
// Each is monotone in its integer numerator for a fixed denominator, so the
// host evaluates the SAME long double expression (same libm, same host
// architecture as the reference) to find the smallest passing integer per
// denominator; the device then compares integers only.
#pragma once
#include <stdint.h>
#include <math.h>
#include <vector>
#include <algorithm>
#include "../../include/imsame_dev.h"

// smallest raw with e(raw) < min_e for this read length (~0: never)
static inline uint64_t imsame_minraw(uint64_t ylen, uint64_t Ldb, long double min_e) {
    auto pass = [&](uint64_t raw) {
        const long double e = (long double)0.333 * (long double)ylen * (long double)Ldb * expl(-0.275 * (long double)raw);
        return e < min_e;
    };
    if (!pass(~0ull)) return ~0ull;
    if (pass(0)) return 0;
    uint64_t lo = 0, hi = ~0ull;                // pass(lo) false, pass(hi) true
    while (hi - lo > 1) {
        const uint64_t m = lo + (hi - lo) / 2;
        if (pass(m)) hi = m; else lo = m;
    }
    return hi;
}

// smallest num in [0, numcap] with (long double)num / den >= thr (~0u: never)
static inline uint32_t imsame_minnum(uint64_t den, long double thr, uint64_t numcap) {
    auto ok = [&](uint64_t num) { return (long double)num / (long double)den >= thr; };
    if (!ok(numcap)) return 0xFFFFFFFFu;
    if (ok(0)) return 0;
    uint64_t lo = 0, hi = numcap;
    while (hi - lo > 1) {
        const uint64_t m = (lo + hi) / 2;
        if (ok(m)) hi = m; else lo = m;
    }
    return (uint32_t)hi;
}

// minraw[ylen], minlen[ylen] for ylen <= ymax; minident[len] for len <= xmax+ymax+1
static inline void imsame_build_tables(const imsame_params *p, uint64_t db_len, uint32_t ymax, uint32_t xmax,
                                       std::vector<uint64_t> &mr, std::vector<uint32_t> &ml,
                                       std::vector<uint32_t> &mi) {
    mr.assign(ymax + 1, 0);
    ml.assign(ymax + 1, 0);
    mi.assign((size_t)xmax + ymax + 2, 0);
    for (uint32_t y = 0; y <= ymax; ++y) {
        mr[y] = imsame_minraw(y, db_len, p->min_e);
        ml[y] = imsame_minnum(y, p->min_coverage, 2ull * (xmax + ymax) + 4);
    }
    for (size_t l = 0; l < mi.size(); ++l) mi[l] = (l == 0) ? 0xFFFFFFFFu : imsame_minnum(l, p->min_identity, l);
}

// int32 safety of the DP (nw_kernel.hip): every score stays within +-2^26
static inline bool imsame_gaps_in_range(int64_t ig, int64_t eg, uint64_t xmax, uint64_t ymax) {
    const long double L = (long double)(xmax + ymax), m = (long double)std::max(xmax, ymax);
    const long double aig = fabsl((long double)ig), aeg = fabsl((long double)eg);
    long double bound;
    if (ig <= 0 && eg <= 0) bound = 4 * L + aig + aeg * m + 8;       // scores never exceed the diagonal
    else bound = L * (4 + aig + aeg * m) + aig + aeg * m + 8;
    return bound < (long double)(1 << 26);
}
