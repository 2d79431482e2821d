// wave_ops.h -- the cross-lane and memory-ordering primitives the kernels use.
//
// On gfx950 they are the hardware ops (DPP wave_shr, ds_bpermute, ballot).
// Under IMSAME_WAVE_EMU (CPU test build only: tests/emu/) every lane of a
// wave is a host thread and each primitive is a lock-step exchange, so the
// very same kernel source runs in the CPU test suite.
#pragma once

#ifndef IMSAME_WAVE_EMU
#include <hip/hip_runtime.h>

#define WV_DEVICE __device__ __forceinline__

// lane l receives lane l-1's value (lane 0 receives 0): DPP wave_shr:1 with
// bound_ctrl zero fill (no v_mov to seed the destination's old value)
WV_DEVICE int wv_shr1(int v) { return __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, true); }
// lane l receives lane l+1's value (lane 63 receives 0): wave_shl:1, zero fill
WV_DEVICE int wv_shl1(int v) { return __builtin_amdgcn_mov_dpp(v, 0x130, 0xf, 0xf, true); }
// lane l receives lane l-1's v, lane 0 its own `fill` (wave_shr:1, bound_ctrl off: old = fill)
WV_DEVICE int wv_shr1_fill(int v, int fill) { return __builtin_amdgcn_update_dpp(fill, v, 0x138, 0xf, 0xf, false); }
// lane l receives lane l+1's v, lane 63 its own `fill` (wave_shl:1)
WV_DEVICE int wv_shl1_fill(int v, int fill) { return __builtin_amdgcn_update_dpp(fill, v, 0x130, 0xf, 0xf, false); }
// max of three signed ints in one VALU op (v_max3_i32)
WV_DEVICE int wv_max3(int a, int b, int c) {
    int r;
    asm("v_max3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
WV_DEVICE unsigned long long wv_ballot(bool p) { return __ballot(p); }
WV_DEVICE bool wv_any(bool p) { return __any(p); }
WV_DEVICE int wv_shfl(int v, int src) { return __shfl(v, src); }
WV_DEVICE int wv_shfl_xor(int v, int m) { return __shfl_xor(v, m); }
WV_DEVICE uint32_t wv_first(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// lane l's v (wave-uniform; every lane must be active)
WV_DEVICE int wv_readlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
WV_DEVICE uint32_t wv_atomic_add(uint32_t *p, uint32_t v) { return atomicAdd(p, v); }
WV_DEVICE void wv_atomic_or(uint32_t *p, uint32_t v) { atomicOr(p, v); }
WV_DEVICE void wv_atomic_min64(unsigned long long *p, unsigned long long v) { atomicMin(p, v); }
WV_DEVICE void wv_atomic_add64(unsigned long long *p, unsigned long long v) { atomicAdd(p, v); }
// shader clock (phase profiling only)
WV_DEVICE unsigned long long wv_clock() { return (unsigned long long)clock64(); }
// the constant 100 MHz counter (s_memrealtime): with wv_clock it gives the shader clock
WV_DEVICE unsigned long long wv_realtime() { return (unsigned long long)__builtin_amdgcn_s_memrealtime(); }
// LDS written by some lanes, read by others of the SAME wave
WV_DEVICE void wv_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// global memory written by some lanes, read by others of the SAME wave
WV_DEVICE void wv_mem_sync() {
    __builtin_amdgcn_s_waitcnt(0);
    __threadfence_block();
}

// Packed pairs: two int16 lanes in one 32-bit register (bits 0-15 = candidate
// A, bits 16-31 = candidate B).  The v_pk_*_i16 forms issue at the same cost
// as one v_max_i32 (scripts/micro/valu_rate.hip), so each does two cells.
typedef short wv_s2 __attribute__((ext_vector_type(2)));
WV_DEVICE wv_s2 pk_v(uint32_t a) { return __builtin_bit_cast(wv_s2, a); }
WV_DEVICE uint32_t pk_u(wv_s2 a) { return __builtin_bit_cast(uint32_t, a); }
WV_DEVICE uint32_t pk_add(uint32_t a, uint32_t b) { return pk_u(pk_v(a) + pk_v(b)); }          // v_pk_add_u16
WV_DEVICE uint32_t pk_sub(uint32_t a, uint32_t b) { return pk_u(pk_v(a) - pk_v(b)); }          // v_pk_sub_u16
WV_DEVICE uint32_t pk_max(uint32_t a, uint32_t b) { return pk_u(__builtin_elementwise_max(pk_v(a), pk_v(b))); }
typedef unsigned short wv_u2 __attribute__((ext_vector_type(2)));
WV_DEVICE uint32_t pk_maxu(uint32_t a, uint32_t b) {                                             // v_pk_max_u16
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(wv_u2, a), __builtin_bit_cast(wv_u2, b)));
}
WV_DEVICE uint32_t pk_minu(uint32_t a, uint32_t b) {                                             // v_pk_min_u16
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(wv_u2, a), __builtin_bit_cast(wv_u2, b)));
}
// 0xFFFF in each half that is negative.  Opaque on purpose: seen as a sign
// splat, LLVM turns the bfi/and_or users into per-half v_cmp + v_cndmask.
WV_DEVICE uint32_t pk_neg_mask(uint32_t a) {
    uint32_t r;
    // op_sel_hi:[0,1]: the high lane takes its shift from the constant's LOW
    // half too (by default it would read bits 16-31 of 15, i.e. 0)
    asm("v_pk_ashrrev_i16 %0, 15, %1 op_sel_hi:[0,1]" : "=v"(r) : "v"(a));
    return r;
}
// (m & c) | w and m ? a : b as v_bitop3_b32 (truth tables 0xEA / 0xCA):
// bitop3 issues at the full VALU rate, v_and_or_b32 / v_bfi_b32 at half
// (scripts/micro/valu_rate.hip); asm so LLVM cannot pick the slow forms.
WV_DEVICE uint32_t wv_and_or(uint32_t m, uint32_t c, uint32_t w) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xea" : "=v"(r) : "v"(m), "v"(c), "v"(w));
    return r;
}
WV_DEVICE uint32_t wv_bfi(uint32_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}
// byte permute of the 8 bytes {hi:lo}: selector byte k picks byte sel_k (0-3 of lo, 4-7 of hi)
WV_DEVICE uint32_t wv_perm(uint32_t hi, uint32_t lo, uint32_t sel) { return __builtin_amdgcn_perm(hi, lo, sel); }
// the 32 bits of {hi:lo} from bit s up (s < 32): one v_alignbit_b32
WV_DEVICE uint32_t wv_alignbit(uint32_t hi, uint32_t lo, uint32_t s) { return __builtin_amdgcn_alignbit(hi, lo, s); }
WV_DEVICE uint32_t wv_bitrev(uint32_t v) { return __builtin_bitreverse32(v); }        // v_bfrev_b32
// (w << 1) | c in one v_addc_co_u32 (w + w + carry): the compare's lane mask
// is the carry-in
WV_DEVICE uint32_t wv_shift_in(uint32_t w, bool c) {
    uint32_t r;
    unsigned long long co;
    asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(co) : "v"(w), "s"(__builtin_amdgcn_ballot_w64(c)));
    return r;
}

#else  // ---------------------------------------------------------- CPU emu
#include <stdint.h>
#include <string.h>
#include <climits>
#include <algorithm>
#include <atomic>

#define WV_DEVICE inline
#define __host__
#define __device__
#define __global__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __restrict__
using std::max;
using std::min;
struct uint2 { uint32_t x, y; };
inline uint2 make_uint2(uint32_t x, uint32_t y) { return uint2{x, y}; }

namespace wvemu {
struct Wave;
extern thread_local Wave *t_wave;
extern thread_local int t_lane;
void sync();                       // all 64 lanes of t_wave
extern thread_local uint64_t *t_xch;
}

inline int wv_lane() { return wvemu::t_lane; }
inline int __mul24(int a, int b) { return a * b; }
inline int wv_max3(int a, int b, int c) { return std::max(a, std::max(b, c)); }
inline int wv_shr1(int v) {
    wvemu::t_xch[wvemu::t_lane] = (uint64_t)(uint32_t)v;
    wvemu::sync();
    int r = wvemu::t_lane ? (int)(uint32_t)wvemu::t_xch[wvemu::t_lane - 1] : 0;
    wvemu::sync();
    return r;
}
inline int wv_shl1(int v) {
    wvemu::t_xch[wvemu::t_lane] = (uint64_t)(uint32_t)v;
    wvemu::sync();
    int r = wvemu::t_lane < 63 ? (int)(uint32_t)wvemu::t_xch[wvemu::t_lane + 1] : 0;
    wvemu::sync();
    return r;
}
inline int wv_shr1_fill(int v, int fill) {
    wvemu::t_xch[wvemu::t_lane] = (uint64_t)(uint32_t)v;
    wvemu::sync();
    int r = wvemu::t_lane ? (int)(uint32_t)wvemu::t_xch[wvemu::t_lane - 1] : fill;
    wvemu::sync();
    return r;
}
inline int wv_shl1_fill(int v, int fill) {
    wvemu::t_xch[wvemu::t_lane] = (uint64_t)(uint32_t)v;
    wvemu::sync();
    int r = wvemu::t_lane < 63 ? (int)(uint32_t)wvemu::t_xch[wvemu::t_lane + 1] : fill;
    wvemu::sync();
    return r;
}
inline unsigned long long wv_ballot(bool p) {
    wvemu::t_xch[wvemu::t_lane] = p;
    wvemu::sync();
    unsigned long long m = 0;
    for (int l = 0; l < 64; ++l) m |= (unsigned long long)(wvemu::t_xch[l] & 1) << l;
    wvemu::sync();
    return m;
}
inline bool wv_any(bool p) { return wv_ballot(p) != 0; }
inline int wv_shfl(int v, int src) {
    wvemu::t_xch[wvemu::t_lane] = (uint64_t)(uint32_t)v;
    wvemu::sync();
    int r = (int)(uint32_t)wvemu::t_xch[((src % 64) + 64) % 64];
    wvemu::sync();
    return r;
}
inline int wv_shfl_xor(int v, int m) { return wv_shfl(v, wvemu::t_lane ^ m); }
inline uint32_t wv_first(uint32_t v) { return (uint32_t)wv_shfl((int)v, 0); }
inline int wv_readlane(int v, int l) { return wv_shfl(v, l); }
inline uint32_t wv_atomic_add(uint32_t *p, uint32_t v) {
    return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST);
}
inline void wv_atomic_or(uint32_t *p, uint32_t v) { __atomic_fetch_or(p, v, __ATOMIC_SEQ_CST); }
inline void wv_atomic_min64(unsigned long long *p, unsigned long long v) {
    unsigned long long cur = __atomic_load_n(p, __ATOMIC_SEQ_CST);
    while (v < cur && !__atomic_compare_exchange_n(p, &cur, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {}
}
inline void wv_atomic_add64(unsigned long long *p, unsigned long long v) { __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST); }
inline unsigned long long wv_clock() { return 0; }
inline unsigned long long wv_realtime() { return 0; }
inline void wv_lds_sync() { wvemu::sync(); }
inline void wv_mem_sync() { wvemu::sync(); }

inline uint32_t pk_map(uint32_t a, uint32_t b, int (*f)(int, int)) {
    const int lo = f((int16_t)(a & 0xFFFF), (int16_t)(b & 0xFFFF)), hi = f((int16_t)(a >> 16), (int16_t)(b >> 16));
    return ((uint32_t)(uint16_t)lo) | ((uint32_t)(uint16_t)hi << 16);
}
inline uint32_t pk_add(uint32_t a, uint32_t b) { return pk_map(a, b, [](int x, int y) { return x + y; }); }
inline uint32_t pk_sub(uint32_t a, uint32_t b) { return pk_map(a, b, [](int x, int y) { return x - y; }); }
inline uint32_t pk_max(uint32_t a, uint32_t b) { return pk_map(a, b, [](int x, int y) { return x > y ? x : y; }); }
inline uint32_t pk_maxu(uint32_t a, uint32_t b) {
    const uint32_t lo = std::max(a & 0xFFFFu, b & 0xFFFFu), hi = std::max(a >> 16, b >> 16);
    return lo | (hi << 16);
}
inline uint32_t pk_minu(uint32_t a, uint32_t b) {
    const uint32_t lo = std::min(a & 0xFFFFu, b & 0xFFFFu), hi = std::min(a >> 16, b >> 16);
    return lo | (hi << 16);
}
inline uint32_t pk_neg_mask(uint32_t a) { return pk_map(a, 0, [](int x, int) { return x < 0 ? -1 : 0; }); }
inline uint32_t wv_shift_in(uint32_t w, bool c) { return (w << 1) | (c ? 1u : 0u); }
inline uint32_t wv_and_or(uint32_t m, uint32_t c, uint32_t w) { return (m & c) | w; }
inline uint32_t wv_bfi(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }
inline uint32_t wv_alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (s & 31));
}
inline uint32_t wv_bitrev(uint32_t v) {
    uint32_t r = 0;
    for (int k = 0; k < 32; ++k) r |= ((v >> k) & 1u) << (31 - k);
    return r;
}
inline uint32_t wv_perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int k = 0; k < 4; ++k) {
        const uint32_t s = (sel >> (8 * k)) & 0xFF;
        uint32_t b;
        if (s < 8) b = (uint32_t)(v >> (8 * s)) & 0xFF;
        else if (s == 12) b = 0;
        else if (s > 12) b = 0xFF;
        else b = ((v >> (s == 8 ? 15 : s == 9 ? 31 : s == 10 ? 47 : 63)) & 1) ? 0xFF : 0;
        r |= b << (8 * k);
    }
    return r;
}
#endif
