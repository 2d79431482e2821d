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

// lane l receives lane l-1's value (lane 0 receives 0): DPP wave_shr:1
WV_DEVICE int wv_shr1(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, false); }
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
WV_DEVICE uint32_t wv_atomic_add(uint32_t *p, uint32_t v) { return atomicAdd(p, v); }
WV_DEVICE void wv_atomic_or(uint32_t *p, uint32_t v) { atomicOr(p, v); }
WV_DEVICE void wv_atomic_min64(unsigned long long *p, unsigned long long v) { atomicMin(p, v); }
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
inline uint32_t wv_atomic_add(uint32_t *p, uint32_t v) {
    return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST);
}
inline void wv_atomic_or(uint32_t *p, uint32_t v) { __atomic_fetch_or(p, v, __ATOMIC_SEQ_CST); }
inline void wv_atomic_min64(unsigned long long *p, unsigned long long v) {
    unsigned long long cur = __atomic_load_n(p, __ATOMIC_SEQ_CST);
    while (v < cur && !__atomic_compare_exchange_n(p, &cur, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {}
}
inline void wv_lds_sync() { wvemu::sync(); }
inline void wv_mem_sync() { wvemu::sync(); }
#endif
