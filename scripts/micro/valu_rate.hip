// valu_rate.hip -- measured VALU issue cost of the instruction forms the NW
// sweep (nw_kernel.hip) is built from, on gfx950.  DESIGN.md prices the
// sweep with these numbers.
//
//   hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip && ./valu_rate
//
// Each kernel runs ITER iterations of 8 independent chains of one
// instruction form; waves per SIMD is set by the grid (4-wave blocks, one
// per SIMD).  Prints SIMD cycles per wave-instruction (clock from
// s_memtime / s_memrealtime), so 2.0 = the 64-lane/2-cycle issue peak.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITER 8192
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

#define K8(stmt) _Pragma("unroll") for (int i = 0; i < 8; ++i) { stmt; }

template <int KIND>
__global__ __launch_bounds__(256) void k_rate(int *out, int seed, unsigned long long *clk) {
    int a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * (i + 1);
    const int b = seed * 3 + threadIdx.x, c = seed ^ 0x55;
    unsigned long long m = 0x5555aaaa3333ccccull ^ (unsigned long long)seed;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0 && blockIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int it = 0; it < ITER; ++it) {
        if (KIND == 0) K8(asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 1) K8(asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 2) K8(asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c)))
        if (KIND == 3) K8(asm volatile("v_max_i32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 4) K8(asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "s"(m)))
        if (KIND == 5) K8(asm volatile("v_cndmask_b32_e64 %0, 0, 4, %1" : "=v"(a[i]) : "s"(m ^ (unsigned)i)))
        if (KIND == 6) K8(asm volatile("v_cmp_gt_i32_e64 %0, %1, %2" : "=s"(m) : "v"(a[i]), "v"(b)))
        if (KIND == 7) K8(asm volatile("v_cmp_gt_i32_e32 vcc, %0, %1" : : "v"(a[i]), "v"(b) : "vcc"))
        if (KIND == 8) K8(asm volatile("s_mov_b64 vcc, %1\n\tv_cndmask_b32_e32 %0, %0, %2, vcc" : "+v"(a[i]) : "s"(m), "v"(b) : "vcc"))
        if (KIND == 9) K8(asm volatile("s_mov_b64 vcc, %1\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc" : "+v"(a[i]) : "s"(m) : "vcc"))
        if (KIND == 10) K8(asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c)))
        if (KIND == 11) K8(asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 12) K8(asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(a[i]) : "v"(a[(i + 4) & 7])))
        if (KIND == 13) K8(asm volatile("v_sub_u32_e32 %0, %1, %0\n\tv_max_i32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 14) K8(asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 15) K8(asm volatile("v_cmp_eq_u32_sdwa %0, %1, %2 src0_sel:BYTE_1 src1_sel:DWORD" : "=s"(m) : "v"(a[i]), "v"(b)))
        if (KIND == 16) K8(asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c)))
        if (KIND == 17) K8(asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c)))
        if (KIND == 18) K8(asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 19) K8(asm volatile("v_pk_sub_i16 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 20) K8(asm volatile("v_pk_ashrrev_i16 %0, 15, %0" : "+v"(a[i])))
        if (KIND == 21) K8(asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a[i]) : "v"(b), "v"(c)))
        if (KIND == 22) K8(asm volatile("v_and_or_b32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c)))
        if (KIND == 23) K8(asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c)))
        if (KIND == 24) K8(asm volatile("v_xor_b32_e32 %0, %1, %0" : "+v"(a[i]) : "v"(b)))
        if (KIND == 25) K8(asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 26) K8(asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a[0]) : "v"(b)))
        if (KIND == 27) K8(asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(a[0]) : "v"(b)))
        if (KIND == 28) K8(asm volatile("v_pk_mad_i16 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c)))
        if (KIND == 29) K8(asm volatile("v_sub_u32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 30) K8(asm volatile("v_lshrrev_b32_e32 %0, 3, %0" : "+v"(a[i])))
        if (KIND == 31) K8(asm volatile("v_or_b32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 32) K8(asm volatile("v_and_b32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 33) K8(asm volatile("v_mov_b32_e32 %0, %1" : "=v"(a[i]) : "v"(a[(i + 1) & 7])))
        if (KIND == 34) K8(asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b) : "vcc"))
        if (KIND == 35) K8(asm volatile("v_max_u16_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 36) K8(asm volatile("v_add_u16_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 37) K8(asm volatile("v_max_f32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 38) K8(asm volatile("v_add_f32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 39) K8(asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(*(double *)&a[i & 6]) : "v"(*(double *)&a[(i + 2) & 6])))
        if (KIND == 40) K8(asm volatile("v_bfe_u32 %0, %0, 3, 5" : "+v"(a[i])))
        if (KIND == 41) K8(asm volatile("v_lshlrev_b32_e32 %0, 3, %0" : "+v"(a[i])))
        if (KIND == 42) K8(asm volatile("v_ashrrev_i32_e32 %0, 3, %0" : "+v"(a[i])))
        if (KIND == 43) K8(asm volatile("v_subrev_u32_e32 %0, %1, %0" : "+v"(a[i]) : "v"(b)))
        if (KIND == 44) K8(asm volatile("v_min_u32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 45) K8(asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(a[i]) : "v"(b), "v"(c)))
        if (KIND == 46) K8(asm volatile("v_add_u32_e32 %0, %0, %1\n\tv_pk_max_i16 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 47) K8(asm volatile("v_sub_u32_dpp %0, %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[i]) : "v"(a[(i + 4) & 7])))
        if (KIND == 48) K8(asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b)))
        if (KIND == 49) K8(asm volatile("v_not_b32_e32 %0, %0" : "+v"(a[i])))
        if (KIND == 50) K8(asm volatile("v_pk_max_i16 %0, %0, %1\n\tv_add_u32_e32 %0, %0, %1\n\tv_sub_u32_e32 %0, %0, %2" : "+v"(a[i]) : "v"(b), "v"(c)))
        if (KIND == 51) K8(asm volatile("v_pk_max_i16 %0, %0, %1\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(a[i]) : "v"(b), "v"(c)))
        if (KIND == 52) K8(asm volatile("v_pk_max_i16 %0, %0, %1\n\tv_pk_add_u16 %0, %0, %2\n\tv_add_u32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(b), "v"(c)))
        if (KIND == 53) K8(asm volatile("v_add_u32_e32 %0, %0, %1\n\tv_sub_u32_e32 %0, %0, %2" : "+v"(a[i]) : "v"(b), "v"(c)))
        if (KIND == 54) K8(asm volatile("v_bfi_b32 %0, %1, %0, %2\n\tv_pk_max_i16 %0, %0, %1" : "+v"(a[i]) : "v"(b), "v"(c)))
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    int s = (int)m;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND>
static int run(const char *name, int ninstr, int *d_out, unsigned long long *d_clk, int cus) {
    printf("%-40s", name);
    for (int wps = 1; wps <= 8; wps *= 2) {              // waves per SIMD
        const int blocks = cus * wps;
        hipEvent_t e0, e1;
        CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
        hipLaunchKernelGGL(k_rate<KIND>, dim3(blocks), dim3(256), 0, 0, d_out, 7, d_clk);
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_rate<KIND>, dim3(blocks), dim3(256), 0, 0, d_out, 7, d_clk);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        unsigned long long clk[2];
        CHK(hipMemcpy(clk, d_clk, sizeof clk, hipMemcpyDeviceToHost));
        const double ghz = (double)clk[0] / ((double)clk[1] / 100e6) / 1e9;
        const double winstr = (double)wps * ITER * 8 * ninstr;                // per SIMD
        printf("  w%d %5.2f", wps, ms * 1e-3 * ghz * 1e9 / winstr);
        CHK(hipEventDestroy(e0)); CHK(hipEventDestroy(e1));
    }
    printf("   cyc/instr/SIMD\n");
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("%s  CUs %d\n", p.gcnArchName, cus);
    int *d_out; unsigned long long *d_clk;
    CHK(hipMalloc(&d_out, (size_t)cus * 8 * 256 * sizeof(int)));
    CHK(hipMalloc(&d_clk, 16));
#define R(K, N, S) if (run<K>(S, N, d_out, d_clk, cus)) return 1;
    R(0, 1, "v_add_u32_e32")
    R(1, 1, "v_add_u32_e64")
    R(2, 1, "v_max3_i32")
    R(3, 1, "v_max_i32_e32")
    R(4, 1, "v_cndmask_b32_e64 (sgpr mask)")
    R(5, 1, "v_cndmask_b32_e64 0,4 (const)")
    R(6, 1, "v_cmp_gt_i32_e64 (-> sgpr)")
    R(7, 1, "v_cmp_gt_i32_e32 (-> vcc)")
    R(8, 1, "s_mov vcc + v_cndmask_b32_e32 [valu only]")
    R(9, 1, "s_mov vcc + v_addc_co_u32_e32 [valu only]")
    R(10, 1, "v_or3_b32")
    R(11, 1, "v_lshl_or_b32")
    R(12, 1, "v_mov_b32_dpp wave_shr:1")
    R(13, 2, "v_sub_u32_e32 + v_max_i32_e32")
    R(14, 1, "v_pk_max_i16")
    R(15, 1, "v_cmp_eq_u32_sdwa")
    R(16, 1, "v_add3_u32")
    R(17, 1, "v_mad_u32_u24")
    R(18, 1, "v_pk_add_u16")
    R(19, 1, "v_pk_sub_i16")
    R(20, 1, "v_pk_ashrrev_i16")
    R(21, 1, "v_bfi_b32")
    R(22, 1, "v_and_or_b32")
    R(23, 1, "v_perm_b32")
    R(24, 1, "v_xor_b32_e32")
    R(25, 1, "v_pk_min_u16")
    R(26, 1, "v_pk_max_i16 (one dependent chain)")
    R(27, 1, "v_add_u32 (one dependent chain)")
    R(28, 1, "v_pk_mad_i16")
    R(29, 1, "v_sub_u32_e32")
    R(30, 1, "v_lshrrev_b32_e32")
    R(31, 1, "v_or_b32_e32")
    R(32, 1, "v_and_b32_e32")
    R(33, 1, "v_mov_b32_e32")
    R(34, 1, "v_cndmask_b32_e32 (vcc)")
    R(35, 1, "v_max_u16_e32")
    R(36, 1, "v_add_u16_e32")
    R(37, 1, "v_max_f32_e32")
    R(38, 1, "v_add_f32_e32")
    R(39, 1, "v_pk_add_f32")
    R(40, 1, "v_bfe_u32")
    R(41, 1, "v_lshlrev_b32_e32")
    R(42, 1, "v_ashrrev_i32_e32")
    R(43, 1, "v_subrev_u32_e32")
    R(44, 1, "v_min_u32_e32")
    R(45, 1, "v_bitop3_b32")
    R(46, 2, "v_add_u32 + v_pk_max_i16 (mixed)")
    R(47, 1, "v_sub_u32_dpp wave_shr:1")
    R(48, 1, "v_pk_max_u16")
    R(49, 1, "v_not_b32_e32")
    R(50, 3, "pk_max + add + sub (mixed)")
    R(51, 2, "pk_max + bitop3 (mixed)")
    R(52, 3, "pk_max + pk_add + add (mixed)")
    R(53, 2, "add + sub (full-rate pair)")
    R(54, 2, "bfi + pk_max (half-rate pair)")
    return 0;
}
