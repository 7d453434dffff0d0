// Standalone timing probe of the tournament narrow-block kernels (tslu.hip),
// built with TSLU_PROBE: s_memtime stamps at fixed points of the tree kernel
// (leaf workgroup 0 and the node of every level).  Not part of the library.
//   hipcc -O3 --offload-arch=gfx950 -DTSLU_PROBE -Icsrc/include -Icsrc/kernels csrc/tools/tslu_probe.hip
//   ./tslu_probe M [reps]
#define TSLU_PROBE 1
#include "../kernels/tslu.hip"

#include <cstdio>
#include <random>
#include <vector>

using namespace slate_amd::dev;

int main(int argc, char** argv) {
    const int64_t m = argc > 1 ? atoll(argv[1]) : 32768;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const int64_t ncols = argc > 3 ? atoll(argv[3]) : 32;
    const int nn = 32;
    std::vector<double> h(m * ncols);
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> U(-1, 1);
    for (auto& x : h) x = U(g);
    double* A;
    int64_t *ipiv, *perm, *work;
    int* info;
    const int64_t wsz = tslu_workspace(m);
    (void)hipMalloc(&A, h.size() * 8);
    (void)hipMalloc(&ipiv, m * 8);
    (void)hipMalloc(&perm, m * 8);
    (void)hipMalloc(&work, wsz * 8);
    (void)hipMalloc(&info, 4);
    hipStream_t s;
    hipStreamCreate(&s);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // SLATE_TSLU_V1 is read once per process: run the probe twice to compare
    for (int v = 0; v < 1; ++v) {
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice);
            hipMemset(info, 0, 4);
            tslu_init(work, s);
            hipStreamSynchronize(s);
            hipEventRecord(e0, s);
            tslu_narrow<double>(m, 0, nn, A, A, m, ncols, ipiv, perm, info, 0, work, s);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = std::min(best, ms);
        }
        printf("%s m=%ld ncols=%ld: best %.1f us\n", getenv("SLATE_TSLU_V1") ? "v1" : "v2", (long)m, (long)ncols, best * 1e3);
    }
    // probe stamps of one more run
    long long zero[128] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_tslu_probe), zero, sizeof(zero));
    hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    tslu_narrow<double>(m, 0, nn, A, A, m, ncols, ipiv, perm, info, 0, work, s);
    hipStreamSynchronize(s);
    long long t[128];
    hipMemcpyFromSymbol(t, HIP_SYMBOL(g_tslu_probe), sizeof(t));
    const char* nm[14] = {"loaded", "k0", "k1", "k2", "k3", "k4", "k5", "k6", "k7", "k16", "k31", "loop", "root-end", "handoff"};
    for (int lv = 0; lv < 4; ++lv) {
        long long b = t[lv * 32];
        if (!b) continue;
        printf("level %d (cycles from 'loaded'):", lv);
        for (int q = 1; q < 14; ++q)
            if (t[lv * 32 + q]) printf(" %s=%lld", nm[q], t[lv * 32 + q] - b);
        printf("\n");
    }
    const char* sn[7] = {"key", "wmax", "publish", "barrier", "read-u", "tn", "update"};
    for (int lv = 0; lv < 4; ++lv)
        for (int kk = 0; kk < 2; ++kk) {
            long long* q = t + lv * 32 + 16 + 8 * kk;
            if (!q[0]) continue;
            printf("level %d step %d sub-steps (cycles from 'key'):", lv, kk ? 20 : 4);
            for (int u = 1; u < 7; ++u) printf(" %s=%lld", sn[u], q[u] - q[0]);
            printf("\n");
        }
    return 0;
}
