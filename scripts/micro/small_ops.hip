// Latency of the small stream operations of a round (counter resets and
// read-backs) while other work holds every wave slot of the chip -- the
// state of a lane's round transitions while the other lanes' NW launches
// run.  A "hog" launch of long-running waves (256 VGPRs: 2
// per SIMD, as nw16's 19-column form) keeps the chip full for ~hog_ms; on a
// second stream each small operation is enqueued and timed from the host:
//   memset 8 B (hipMemsetAsync), D2H 24 B into pageable / pinned memory,
//   H2D 8 B from pinned memory, a 1-block kernel.
// Each is timed alone first (idle chip), then under the hog.  Output: one
// JSON line.  Measurement only.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#include <string>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e)); return 1; } } while (0)

// every wave spins until `ticks` of the 100 MHz real-time counter have passed
// since it started: the chip's slots stay held for that long (a bounded loop:
// every wave exits)
__global__ __launch_bounds__(256) void hog(float *out, int ticks) {
    float a = threadIdx.x, b = blockIdx.x;
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < (unsigned long long)ticks) {
        for (int i = 0; i < 64; ++i) { a = a * 1.000001f + b; b = b * 0.999999f + a; }
    }
    if (a == -1.f) out[0] = b;
}
__global__ void one(unsigned *p) { if (threadIdx.x == 0) p[0] += 1; }

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000000;     // 20 ms per wave
    hipStream_t sh, ss;
    CK(hipStreamCreateWithFlags(&sh, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking));
    float *fo; unsigned *dc;
    CK(hipMalloc(&fo, 4)); CK(hipMalloc(&dc, 256));
    unsigned *pin; CK(hipHostMalloc((void **)&pin, 256, hipHostMallocDefault));
    unsigned pageable[64];
    int ncu = 0; CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int blocks = ncu * 8 * 2;            // 8 waves per CU per block-of-4 x 2: every slot, twice over
    auto op = [&](const std::string &k) -> int {
        if (k == "memset") return hipMemsetAsync(dc, 0, 8, ss) != hipSuccess;
        if (k == "d2h_pageable") return hipMemcpyAsync(pageable, dc, 24, hipMemcpyDeviceToHost, ss) != hipSuccess;
        if (k == "d2h_pinned") return hipMemcpyAsync(pin, dc, 24, hipMemcpyDeviceToHost, ss) != hipSuccess;
        if (k == "h2d_pinned") return hipMemcpyAsync(dc, pin, 8, hipMemcpyHostToDevice, ss) != hipSuccess;
        if (k == "kernel1") { one<<<1, 64, 0, ss>>>(dc); return hipGetLastError() != hipSuccess; }
        if (k == "writevalue") return hipStreamWriteValue64(ss, dc, 0, 0) != hipSuccess;
        if (k == "d2h_pinned_4k") return hipMemcpyAsync(pin, dc, 256, hipMemcpyDeviceToHost, ss) != hipSuccess;
        return 1;
    };
    const char *ops[] = {"memset", "writevalue", "d2h_pageable", "d2h_pinned", "d2h_pinned_4k", "h2d_pinned", "kernel1"};
    // hog alone
    double t0 = now_us();
    hog<<<blocks, 256, 0, sh>>>(fo, iters);
    CK(hipStreamSynchronize(sh));
    const double hog_us = now_us() - t0;
    printf("{\"ncu\": %d, \"hog_ms\": %.3f", ncu, hog_us / 1e3);
    for (const char *k : ops) {
        std::vector<double> idle, busy;
        for (int r = 0; r < 5; ++r) {
            double a = now_us();
            if (op(k)) return 1;
            CK(hipStreamSynchronize(ss));
            idle.push_back(now_us() - a);
        }
        for (int r = 0; r < 3; ++r) {
            hog<<<blocks, 256, 0, sh>>>(fo, iters);
            double w = now_us();
            while (now_us() - w < 3000) {}       // the hog's waves hold the slots
            double a = now_us();
            if (op(k)) return 1;
            CK(hipStreamSynchronize(ss));
            busy.push_back(now_us() - a);
            CK(hipStreamSynchronize(sh));
        }
        std::sort(idle.begin(), idle.end()); std::sort(busy.begin(), busy.end());
        printf(", \"%s_idle_us\": %.1f, \"%s_busy_us\": [%.1f, %.1f, %.1f]", k, idle[2], k, busy[0], busy[1], busy[2]);
    }
    printf("}\n");
    return 0;
}
