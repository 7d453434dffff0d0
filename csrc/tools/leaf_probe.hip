// Standalone timing probe of the blocked potrf leaf kernel (aux.hip), built
// with LEAF_PROBE: clock64 stamps after the loads, the factor, the A21 loads,
// the solve and the stores, per workgroup.  Not part of the library.
//   hipcc -O3 --offload-arch=gfx950 -DLEAF_PROBE -Icsrc/include -Icsrc/kernels csrc/tools/leaf_probe.hip
//   ./leaf_probe [r] [reps]
#define LEAF_PROBE 1
#include "../kernels/aux.hip"

#include <cstdio>
#include <random>
#include <vector>

using namespace slate_amd::dev;

int main(int argc, char** argv) {
    const int64_t r = argc > 1 ? atoll(argv[1]) : 448;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const int b = 64;
    const int64_t n = b + r, lda = n;
    std::vector<double> h(n * n);
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> U(-1, 1);
    for (auto& x : h) x = U(g) * 0.01;
    for (int64_t j = 0; j < n; ++j) h[j + j * lda] += 1.0;
    for (int64_t j = 0; j < n; ++j)      // symmetric
        for (int64_t i = 0; i < j; ++i) h[i + j * lda] = h[j + i * lda];
    double *A, *W;
    int* info;
    (void)hipMalloc(&A, h.size() * 8);
    (void)hipMalloc(&W, 64 * 64 * 8);
    (void)hipMalloc(&info, 4);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int k = 0; k < reps; ++k) {
        (void)hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice);
        (void)hipMemset(info, 0, 4);
        (void)hipStreamSynchronize(s);
        (void)hipEventRecord(e0, s);
        potrf_leaf<double>(b, r, A, lda, info, 0, W, nullptr, nullptr, 0, s);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = std::min(best, ms);
    }
    int hinfo = -1;
    (void)hipMemcpy(&hinfo, info, 4, hipMemcpyDeviceToHost);
    long long st[64 * 8];
    (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(g_leaf_probe), sizeof(st));
    printf("leaf b=64 r=%ld: best %.1f us, info %d \n", (long)r, best * 1e3, hinfo);
    const char* names[] = {"load a", "factor", "(wg0 store) / sync+load y", "solve", "store y"};
    for (int w : {0, 1}) {
        if (w == 1 && r == 0) break;
        printf("  wg %d:", w);
        for (int k = 0; k < 5; ++k) {
            if (w == 0 && k >= 2) break;
            printf("  %s %lld", names[k], st[w * 8 + k + 1] - st[w * 8 + k]);
        }
        printf("\n");
    }
    // small triangular solve (LU panel U12 solves): m = 64 unit lower, 448 columns
    {
        const int64_t nc = 448;
        float bt = 1e30f;
        for (int k = 0; k < reps; ++k) {
            (void)hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice);
            (void)hipStreamSynchronize(s);
            (void)hipEventRecord(e0, s);
            trsm_small<double>('L', 'U', 64, nc, A, lda, A + 64 * lda, lda, s);
            (void)hipEventRecord(e1, s);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            bt = std::min(bt, ms);
        }
        (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(g_leaf_probe), sizeof(st));
        const char* tn[] = {"load triangle", "load B", "y from LDS", "solve", "store"};
        printf("trsm_small m=64 n=%ld: best %.1f us\n  wg 0:", (long)nc, bt * 1e3);
        for (int k = 0; k < 5; ++k) printf("  %s %lld", tn[k], st[k + 1] - st[k]);
        printf("\n");
    }
    return 0;
}
