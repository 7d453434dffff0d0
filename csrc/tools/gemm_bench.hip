// Standalone GEMM check + timing harness (development tool, not the product).
// Usage: gemm_bench [m n k] ; checks every transpose combination on odd
// shapes against a naive device reference, then times large square fp64/fp32.
#include "../kernels/device_common.hh"
#include "../kernels/kernels.hh"
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <chrono>
#include <algorithm>
#include <string>

using namespace slate_amd::dev;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

template <typename T>
__global__ void ref_gemm(char ta, char tb, int64_t m, int64_t n, int64_t k, T alpha,
                         const T* A, int64_t lda, const T* B, int64_t ldb, T beta, T* C, int64_t ldc) {
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    int64_t j = blockIdx.y;
    if (i >= m || j >= n) return;
    double s = 0;
    for (int64_t l = 0; l < k; ++l) {
        double a = (ta == 'N') ? A[i + l * lda] : A[l + i * lda];
        double b = (tb == 'N') ? B[l + j * ldb] : B[j + l * ldb];
        s += a * b;
    }
    C[i + j * ldc] = T(alpha * s + (double)beta * (double)C[i + j * ldc]);
}

__global__ void fill(double* p, int64_t n, uint64_t seed) {
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) {
        uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
        x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
        p[i] = (double)(x >> 11) / (double)(1ull << 53) * 2.0 - 1.0;
    }
}
__global__ void tofloat(const double* s, float* d, int64_t n) {
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) d[i] = (float)s[i];
}

template <typename T>
double check(char ta, char tb, int64_t m, int64_t n, int64_t k, int64_t pad) {
    int64_t am = ta == 'N' ? m : k, an = ta == 'N' ? k : m;
    int64_t bm = tb == 'N' ? k : n, bn = tb == 'N' ? n : k;
    int64_t lda = am + pad, ldb = bm + pad, ldc = m + pad;
    double *dA, *dB, *dC;
    CHECK(hipMalloc(&dA, lda * an * 8)); CHECK(hipMalloc(&dB, ldb * bn * 8)); CHECK(hipMalloc(&dC, ldc * n * 8));
    fill<<<(lda * an + 255) / 256, 256>>>(dA, lda * an, 1);
    fill<<<(ldb * bn + 255) / 256, 256>>>(dB, ldb * bn, 2);
    fill<<<(ldc * n + 255) / 256, 256>>>(dC, ldc * n, 3);
    T *A, *B, *C, *C2;
    CHECK(hipMalloc(&A, lda * an * sizeof(T))); CHECK(hipMalloc(&B, ldb * bn * sizeof(T)));
    CHECK(hipMalloc(&C, ldc * n * sizeof(T))); CHECK(hipMalloc(&C2, ldc * n * sizeof(T)));
    if constexpr (sizeof(T) == 8) {
        CHECK(hipMemcpy(A, dA, lda * an * 8, hipMemcpyDeviceToDevice));
        CHECK(hipMemcpy(B, dB, ldb * bn * 8, hipMemcpyDeviceToDevice));
        CHECK(hipMemcpy(C, dC, ldc * n * 8, hipMemcpyDeviceToDevice));
    } else {
        tofloat<<<(lda * an + 255) / 256, 256>>>(dA, (float*)A, lda * an);
        tofloat<<<(ldb * bn + 255) / 256, 256>>>(dB, (float*)B, ldb * bn);
        tofloat<<<(ldc * n + 255) / 256, 256>>>(dC, (float*)C, ldc * n);
    }
    CHECK(hipMemcpy(C2, C, ldc * n * sizeof(T), hipMemcpyDeviceToDevice));
    T alpha = T(0.7), beta = T(-0.3);
    gemm_real<T>(ta, tb, m, n, k, alpha, A, lda, 0, B, ldb, 0, beta, C, ldc, 0, 1, 0);
    ref_gemm<T><<<dim3((m + 127) / 128, n), 128>>>(ta, tb, m, n, k, alpha, A, lda, B, ldb, beta, C2, ldc);
    CHECK(hipDeviceSynchronize());
    std::vector<T> h1(ldc * n), h2(ldc * n);
    CHECK(hipMemcpy(h1.data(), C, ldc * n * sizeof(T), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(h2.data(), C2, ldc * n * sizeof(T), hipMemcpyDeviceToHost));
    double err = 0;
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < m; ++i)
            err = fmax(err, fabs((double)h1[i + j * ldc] - (double)h2[i + j * ldc]));
    hipFree(dA); hipFree(dB); hipFree(dC); hipFree(A); hipFree(B); hipFree(C); hipFree(C2);
    return err / (double)k;
}

template <typename T>
void timeit(char ta, char tb, int64_t n, int64_t k, int reps, int64_t pad = 0) {
    T *A, *B, *C;
    const int64_t ne = (std::max(n, k) + pad) * std::max(n, k);   // operand storage incl. padded ld
    CHECK(hipMalloc(&A, ne * sizeof(T))); CHECK(hipMalloc(&B, ne * sizeof(T))); CHECK(hipMalloc(&C, (n + pad) * n * sizeof(T)));
    double* tmp; CHECK(hipMalloc(&tmp, ne * 8));
    fill<<<(ne + 255) / 256, 256>>>(tmp, ne, 5);
    if constexpr (sizeof(T) == 8) { CHECK(hipMemcpy(A, tmp, ne * 8, hipMemcpyDeviceToDevice)); CHECK(hipMemcpy(B, tmp, ne * 8, hipMemcpyDeviceToDevice)); }
    else { tofloat<<<(ne + 255) / 256, 256>>>(tmp, (float*)A, ne); tofloat<<<(ne + 255) / 256, 256>>>(tmp, (float*)B, ne); }
    CHECK(hipMemset(C, 0, (n + pad) * n * sizeof(T)));
    int64_t lda = (ta == 'N' ? n : k) + pad, ldb = (tb == 'N' ? k : n) + pad;
    if (getenv("GEMM_LD0")) { lda = 0; ldb = 0; }   // lab: operands always cache-resident
    const int64_t ldc = n + pad;
    gemm_real<T>(ta, tb, n, n, k, T(1), A, lda, 0, B, ldb, 0, T(1), C, ldc, 0, 1, 0);
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r)
        gemm_real<T>(ta, tb, n, n, k, T(1), A, lda, 0, B, ldb, 0, T(1), C, ldc, 0, 1, 0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double tf = 2.0 * n * n * k * reps / (ms * 1e-3) / 1e12;
    printf("%s %c%c n=%ld k=%ld ldpad=%ld : %.3f ms/call  %.2f TFLOP/s\n", sizeof(T) == 8 ? "dgemm" : "sgemm", ta, tb, n, k, pad, ms / reps, tf);
    hipFree(A); hipFree(B); hipFree(C); hipFree(tmp);
}

// trailing-update shapes: general NT / NN and lower-triangle NT (syrk) at n x n x k
void tri_sweep(int64_t n, int64_t k, int reps) {
    double *A, *C;
    CHECK(hipMalloc(&A, n * k * 8)); CHECK(hipMalloc(&C, n * n * 8));
    fill<<<(n * k + 255) / 256, 256>>>(A, n * k, 7);
    CHECK(hipMemset(C, 0, n * n * 8));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](const char* name, double flops, auto&& f) {
        f(); CHECK(hipDeviceSynchronize());
        hipEventRecord(e0);
        for (int r = 0; r < reps; ++r) f();
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("%-10s n=%ld k=%ld : %.3f ms/call %.2f TFLOP/s\n", name, n, k, ms / reps, flops * reps / (ms * 1e-3) / 1e12);
    };
    const double full = 2.0 * n * n * k, half = double(n) * (n + 1) * k;
    run("gemm_NT", full, [&] { gemm_real<double>('N', 'T', n, n, k, -1.0, A, n, 0, A, n, 0, 1.0, C, n, 0, 1, 0); });
    run("tri_L_NT", half, [&] { gemm_tri_real<double>('L', 'N', 'T', n, k, -1.0, A, n, A, n, 1.0, C, n, 0); });
    // B stored K-contiguous (the transposed panel copy): NN form
    double* At; CHECK(hipMalloc(&At, n * k * 8));
    fill<<<(n * k + 255) / 256, 256>>>(At, n * k, 8);
    run("gemm_NN", full, [&] { gemm_real<double>('N', 'N', n, n, k, -1.0, A, n, 0, At, k, 0, 1.0, C, n, 0, 1, 0); });
    run("tri_L_NN", half, [&] { gemm_tri_real<double>('L', 'N', 'N', n, k, -1.0, A, n, At, k, 1.0, C, n, 0); });
    run("gemm_TN", full, [&] { gemm_real<double>('T', 'N', n, n, k, -1.0, At, k, 0, At, k, 0, 1.0, C, n, 0, 1, 0); });
    run("tri_L_TN", half, [&] { gemm_tri_real<double>('L', 'T', 'N', n, k, -1.0, At, k, At, k, 1.0, C, n, 0); });
    hipFree(A); hipFree(At); hipFree(C);
}

// QR trailing-update product W = V^T C (nb x n, K = m): one launch, K-chunked
// launches with beta accumulation, and batched split-K + in-order reduce
void vhc_sweep(int64_t nb, int64_t n, int64_t m, int reps) {
    double *V, *C, *W, *P;
    CHECK(hipMalloc(&V, m * nb * 8)); CHECK(hipMalloc(&C, m * n * 8)); CHECK(hipMalloc(&W, nb * n * 8));
    CHECK(hipMalloc(&P, 16 * nb * n * 8));
    fill<<<(m * nb + 255) / 256, 256>>>(V, m * nb, 3);
    fill<<<(m * n + 255) / 256, 256>>>(C, m * n, 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](const char* name, auto&& f) {
        f(); CHECK(hipDeviceSynchronize());
        hipEventRecord(e0);
        for (int r = 0; r < reps; ++r) f();
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("%-14s nb=%ld n=%ld m=%ld : %.3f ms/call %.2f TFLOP/s\n", name, nb, n, m, ms / reps,
               2.0 * nb * n * m * reps / (ms * 1e-3) / 1e12);
    };
    run("one_launch", [&] { gemm_real<double>('T', 'N', nb, n, m, 1.0, V, m, 0, C, m, 0, 0.0, W, nb, 0, 1, 0); });
    for (int64_t kch : {int64_t(8192), int64_t(4096)}) {
        char name[32]; snprintf(name, sizeof name, "kchunk_%ld", kch);
        run(name, [&] {
            for (int64_t r0 = 0; r0 < m; r0 += kch)
                gemm_real<double>('T', 'N', nb, n, std::min(kch, m - r0), 1.0, V + r0, m, 0, C + r0, m, 0,
                                  r0 ? 1.0 : 0.0, W, nb, 0, 1, 0);
        });
    }
    for (int S : {2, 4, 8, 16}) {
        int64_t kc = (m + S - 1) / S;
        char name[32]; snprintf(name, sizeof name, "splitk_%d", S);
        run(name, [&] {
            gemm_real<double>('T', 'N', nb, n, kc, 1.0, V, m, kc, C, m, kc, 0.0, P, nb, nb * n, S, 0);
            splitk_reduce<double>(nb, n, S, P, 1.0, 0.0, W, nb, 0);
        });
    }
    hipFree(V); hipFree(C); hipFree(W); hipFree(P);
}

int main(int argc, char** argv) {
    const char ops[2] = {'N', 'T'};
    if (argc > 1 && std::string(argv[1]) == "vhc") {   // gemm_bench vhc NB N M [reps]
        vhc_sweep(atoll(argv[2]), atoll(argv[3]), atoll(argv[4]), argc > 5 ? atoi(argv[5]) : 3);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "tri") {   // gemm_bench tri N K [reps]
        int64_t N = atoll(argv[2]), K = atoll(argv[3]);
        tri_sweep(N, K, argc > 4 ? atoi(argv[4]) : 3);
        return 0;
    }
    if (argc > 2) {   // gemm_bench N K pad [reps]: leading-dimension padding study only
        int64_t N = atoll(argv[1]), K = atoll(argv[2]), pad = argc > 3 ? atoll(argv[3]) : 0;
        int reps = argc > 4 ? atoi(argv[4]) : 1;
        timeit<double>('N', 'N', N, K, 1, pad);   // warm
        timeit<double>('N', 'N', N, K, reps, pad);
        timeit<double>('N', 'T', N, K, reps, pad);
        timeit<double>('T', 'N', N, K, reps, pad);
        return 0;
    }
    int64_t shapes[][3] = {{1, 1, 1}, {17, 33, 5}, {128, 128, 16}, {129, 131, 67}, {300, 257, 513}, {1000, 999, 77}};
    bool ok = true;
    for (auto& s : shapes)
        for (char ta : ops) for (char tb : ops) for (int pad = 0; pad < 2; ++pad) {
            double e = check<double>(ta, tb, s[0], s[1], s[2], pad ? 3 : 0);
            double ef = check<float>(ta, tb, s[0], s[1], s[2], pad ? 3 : 0);
            bool good = e < 1e-14 && ef < 1e-5;
            ok &= good;
            if (!good || s[0] == 300)
                printf("check %c%c m=%ld n=%ld k=%ld pad=%d: d err/k=%.3e  s err/k=%.3e %s\n", ta, tb, s[0], s[1], s[2], pad, e, ef, good ? "ok" : "FAIL");
        }
    printf("correctness: %s\n", ok ? "PASS" : "FAIL");
    int64_t N = argc > 1 ? atoll(argv[1]) : 8192;
    timeit<double>('N', 'T', N, 512, 5);
    timeit<double>('N', 'N', N, 512, 5);
    timeit<double>('N', 'N', N, N, 2);
    timeit<double>('T', 'N', N, N, 2);
    timeit<float>('N', 'N', N, N, 2);
    timeit<float>('N', 'T', N, 512, 5);
    return ok ? 0 : 1;
}
