// Shader clock vs constant 100 MHz counter inside one wave: the effective
// engine clock seen by a lone latency-bound wave (panel kernels), and the
// cost of one dependent fp64 FMA / DPP / readlane chain step.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void probe(unsigned long long* out, double* sink, int iters) {
    double x = threadIdx.x * 1e-3, y = 1.000001;
    unsigned long long c0 = __builtin_readcyclecounter();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) x = fma(x, y, 1e-9);           // dependent fp64 FMA chain
    unsigned long long c1 = __builtin_readcyclecounter();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    int v = threadIdx.x;
    for (int i = 0; i < iters; ++i) v = __builtin_amdgcn_update_dpp(v, v, 0x124, 0xF, 0xF, false) + 1;  // DPP chain
    unsigned long long c2 = __builtin_readcyclecounter();
    int w = threadIdx.x;
    for (int i = 0; i < iters; ++i) w = __builtin_amdgcn_readlane(w, i & 63) + 1;   // readlane chain
    unsigned long long c3 = __builtin_readcyclecounter();
    unsigned long long r3 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[0] = c1 - c0; out[1] = r1 - r0; out[2] = c2 - c1; out[3] = c3 - c2; out[4] = r3 - r0; out[5] = c3 - c0;
    }
    sink[threadIdx.x] = x + v + w;
}

int main() {
    unsigned long long* d; double* s;
    hipMalloc(&d, 64); hipMalloc(&s, 64 * 8);
    const int iters = 100000;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, s, iters);
        unsigned long long h[6];
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        double t_us = h[4] / 100.0;   // 100 MHz
        printf("fma chain: %.2f cyc/iter; dpp chain %.2f cyc/iter; readlane chain %.2f cyc/iter; "
               "total %llu cyc in %.1f us -> %.0f MHz\n",
               double(h[0]) / iters, double(h[2]) / iters, double(h[3]) / iters, h[5], t_us, h[5] / t_us);
    }
    return 0;
}
