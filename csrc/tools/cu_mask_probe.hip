// CU-mask placement probe (development tool, not the product).
//
// Question it answers: when a stream is created with hipExtStreamCreateWithCUMask,
// which physical CUs (XCC, SE, CU) does each user-mask bit select, and does a
// trailing-size fp64 GEMM on the complement mask keep (256 - R) / 256 of its
// unmasked rate?  Round 5 reserved bits c % (256 / R) == 0, which the KFD maps
// (bit i -> XCC i mod 8) onto ONE XCD; device.cc now reserves bits 0 .. R-1.
//
// Usage: cu_mask_probe [R ...]   (default 8 16 24 32)
#include "../kernels/device_common.hh"
#include "../kernels/kernels.hh"
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>
#include <vector>

using namespace slate_amd::dev;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

// one wave per block: record where it ran, then spin ~20 us so that the
// dispatcher has to spread the grid over every CU the mask allows
__global__ void where_kernel(uint32_t* out, int spin) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (threadIdx.x == 0) out[blockIdx.x] = (xcc & 0xf) << 16 | (hw & 0xffff);
    uint64_t t0 = __builtin_readcyclecounter();
    while (__builtin_readcyclecounter() - t0 < (uint64_t)spin) __builtin_amdgcn_s_sleep(1);
}

// HW_ID (gfx9): cu_id [11:8], sh_id [12], se_id [15:13]
struct Where { int xcc, se, sh, cu; };
static Where decode(uint32_t v) {
    uint32_t hw = v & 0xffff;
    return {int(v >> 16), int((hw >> 13) & 7), int((hw >> 12) & 1), int((hw >> 8) & 15)};
}

static std::vector<uint32_t> mask_bits(int ncu, int R, bool strided, bool complement) {
    std::vector<uint32_t> m((ncu + 31) / 32, 0);
    int stride = R > 0 ? ncu / R : 1;
    for (int c = 0; c < ncu; ++c) {
        bool res = strided ? (c % stride == 0 && c / stride < R) : (c < R);
        if (res != complement) m[c / 32] |= 1u << (c % 32);
    }
    return m;
}

static void placement(int ncu, int R, bool strided) {
    auto m = mask_bits(ncu, R, strided, false);
    hipStream_t s;
    CHECK(hipExtStreamCreateWithCUMask(&s, uint32_t(m.size() * 32), m.data()));
    const int nb = 4096;
    uint32_t* d;
    CHECK(hipMalloc(&d, nb * 4));
    where_kernel<<<nb, 64, 0, s>>>(d, 20000);
    CHECK(hipStreamSynchronize(s));
    std::vector<uint32_t> h(nb);
    CHECK(hipMemcpy(h.data(), d, nb * 4, hipMemcpyDeviceToHost));
    std::set<std::tuple<int, int, int, int>> cus;
    std::vector<int> per_xcc(16, 0);
    for (uint32_t v : h) {
        Where w = decode(v);
        if (cus.insert({w.xcc, w.se, w.sh, w.cu}).second) per_xcc[w.xcc & 15]++;
    }
    printf("R=%-3d %-9s distinct CUs %3zu  per XCC:", R, strided ? "strided" : "bits0..R", cus.size());
    for (int x = 0; x < 8; ++x) printf(" %d", per_xcc[x]);
    // which shader engines of XCC 0 the selected CUs sit in
    std::vector<int> per_se(8, 0);
    for (auto const& c : cus) if (std::get<0>(c) == 0) per_se[std::get<1>(c) & 7]++;
    printf("  XCC0 per SE:");
    for (int e = 0; e < 4; ++e) printf(" %d", per_se[e]);
    printf("\n");
    CHECK(hipFree(d));
    CHECK(hipStreamDestroy(s));
}

__global__ void fill(double* p, int64_t n) {
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < n) p[i] = double((i * 2654435761u) % 1000) * 1e-3 - 0.5;
}

static double gemm_ms(hipStream_t s, int64_t n, int64_t k, double* A, double* B, double* C, int reps) {
    gemm_real<double>('N', 'T', n, n, k, -1.0, A, n, 0, B, n, 0, 1.0, C, n, 0, 1, s);
    CHECK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r)
        gemm_real<double>('N', 'T', n, n, k, -1.0, A, n, 0, B, n, 0, 1.0, C, n, 0, 1, s);
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    hipEventDestroy(e0); hipEventDestroy(e1);
    return ms / reps;
}

// one-wave kernel: the 100 MHz real-time clock when it starts
__global__ void stamp_kernel(uint64_t* out, int i) {
    if (threadIdx.x == 0) out[i] = __builtin_amdgcn_s_memrealtime();
}

// Does a short kernel on stream B start while a long GEMM occupies stream A?
// For each configuration: GEMM on A (stamp before and after it), then after
// ~2 ms 20 stamps on B, each synchronized from the host.  Prints the B
// stamps relative to the GEMM's start and end.
static void overlap(int ncu, double* A, double* B, double* C) {
    const int64_t n = 16384, k = 4096;
    uint64_t* d;
    CHECK(hipMalloc(&d, 64 * 8));
    int lo, hi;
    CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    struct Cfg { const char* name; int prio_b; int reserve; bool mask_a, mask_b; };
    Cfg cfgs[] = {{"B same priority", lo, 0, false, false},
                  {"B high priority", hi, 0, false, false},
                  {"A masked R=32, B high prio unmasked", hi, 32, true, false},
                  {"A masked R=32, B masked to the 32", lo, 32, true, true}};
    for (auto const& c : cfgs) {
        hipStream_t sa, sb;
        if (c.mask_a) {
            auto m = mask_bits(ncu, c.reserve, false, true);
            CHECK(hipExtStreamCreateWithCUMask(&sa, uint32_t(m.size() * 32), m.data()));
        } else {
            CHECK(hipStreamCreateWithPriority(&sa, hipStreamNonBlocking, lo));
        }
        if (c.mask_b) {
            auto m = mask_bits(ncu, c.reserve, false, false);
            CHECK(hipExtStreamCreateWithCUMask(&sb, uint32_t(m.size() * 32), m.data()));
        } else {
            CHECK(hipStreamCreateWithPriority(&sb, hipStreamNonBlocking, c.prio_b));
        }
        stamp_kernel<<<1, 64, 0, sb>>>(d, 63);   // warm both queues
        CHECK(hipStreamSynchronize(sb));
        CHECK(hipMemset(d, 0, 64 * 8));
        stamp_kernel<<<1, 64, 0, sa>>>(d, 0);
        gemm_real<double>('N', 'T', n, n, k, -1.0, A, n, 0, B, n, 0, 1.0, C, n, 0, 1, sa);
        stamp_kernel<<<1, 64, 0, sa>>>(d, 1);
        auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(2)) {}
        for (int i = 0; i < 20; ++i) {
            stamp_kernel<<<1, 64, 0, sb>>>(d, 2 + i);
            CHECK(hipStreamSynchronize(sb));
        }
        CHECK(hipStreamSynchronize(sa));
        std::vector<uint64_t> h(64);
        CHECK(hipMemcpy(h.data(), d, 64 * 8, hipMemcpyDeviceToHost));
        const double g0 = double(h[0]), us = 0.01;   // 100 MHz ticks -> us
        int inside = 0;
        for (int i = 0; i < 20; ++i) inside += h[2 + i] < h[1];
        printf("%-38s gemm %.2f ms; B stamps at +%.0f .. +%.0f us (first, last), %d of 20 before the GEMM ended\n",
               c.name, (h[1] - h[0]) * us * 1e-3, (h[2] - g0) * us, (h[21] - g0) * us, inside);
        CHECK(hipStreamDestroy(sa));
        CHECK(hipStreamDestroy(sb));
    }
    // is a CU-masked stream blocking (synchronizes with the legacy null stream)?
    {
        auto m = mask_bits(ncu, 32, false, true);
        hipStream_t sa, sn;
        CHECK(hipExtStreamCreateWithCUMask(&sa, uint32_t(m.size() * 32), m.data()));
        CHECK(hipStreamCreateWithPriority(&sn, hipStreamNonBlocking, lo));
        unsigned fa = 0, fn = 0;
        CHECK(hipStreamGetFlags(sa, &fa));
        CHECK(hipStreamGetFlags(sn, &fn));
        printf("stream flags: CU-masked %u, hipStreamNonBlocking-created %u (hipStreamNonBlocking = %u)\n", fa, fn,
               unsigned(hipStreamNonBlocking));
        for (int which = 0; which < 2; ++which) {
            hipStream_t sg = which == 0 ? sa : sn;
            CHECK(hipMemset(d, 0, 64 * 8));
            CHECK(hipDeviceSynchronize());
            stamp_kernel<<<1, 64, 0, sg>>>(d, 0);
            gemm_real<double>('N', 'T', n, n, k, -1.0, A, n, 0, B, n, 0, 1.0, C, n, 0, 1, sg);
            stamp_kernel<<<1, 64, 0, sg>>>(d, 1);
            auto t0 = std::chrono::steady_clock::now();
            while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(2)) {}
            stamp_kernel<<<1, 64, 0, nullptr>>>(d, 2);   // the legacy null stream
            CHECK(hipStreamSynchronize(nullptr));
            CHECK(hipDeviceSynchronize());
            std::vector<uint64_t> h(64);
            CHECK(hipMemcpy(h.data(), d, 64 * 8, hipMemcpyDeviceToHost));
            printf("GEMM on a %s stream: a null-stream kernel issued at +2 ms ran at +%.0f us (GEMM %.0f us) -> %s\n",
                   which == 0 ? "CU-masked" : "non-blocking", (h[2] - double(h[0])) * 0.01, (h[1] - double(h[0])) * 0.01,
                   h[2] > h[1] ? "waited for the GEMM (blocking stream)" : "overlapped");
        }
        CHECK(hipStreamDestroy(sa));
        CHECK(hipStreamDestroy(sn));
    }
    CHECK(hipFree(d));
}

int main(int argc, char** argv) {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    printf("device %s, %d CUs\n", prop.gcnArchName, ncu);
    std::vector<int> Rs;
    for (int i = 1; i < argc; ++i) Rs.push_back(atoi(argv[i]));
    if (Rs.empty()) Rs = {8, 16, 24, 32};

    placement(ncu, ncu, false);   // every bit: the whole device
    for (int R : Rs) { placement(ncu, R, true); placement(ncu, R, false); }

    // trailing-size update: 16384^2 x 512 (one 2x4 rank's block at k ~ 0)
    const int64_t n = 16384, k = 512;
    double *A, *B, *C;
    CHECK(hipMalloc(&A, n * k * 8)); CHECK(hipMalloc(&B, n * k * 8)); CHECK(hipMalloc(&C, n * n * 8));
    fill<<<(n * k + 255) / 256, 256>>>(A, n * k);
    fill<<<(n * k + 255) / 256, 256>>>(B, n * k);
    CHECK(hipMemset(C, 0, n * n * 8));
    hipStream_t s0;
    CHECK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    if (getenv("PROBE_OVERLAP")) {
        double *A4, *B4;
        CHECK(hipMalloc(&A4, n * 4096 * 8)); CHECK(hipMalloc(&B4, n * 4096 * 8));
        fill<<<(n * 4096 + 255) / 256, 256>>>(A4, n * 4096);
        fill<<<(n * 4096 + 255) / 256, 256>>>(B4, n * 4096);
        CHECK(hipDeviceSynchronize());
        overlap(ncu, A4, B4, C);
        return 0;
    }
    const double base = gemm_ms(s0, n, k, A, B, C, 10);
    const double fl = 2.0 * n * n * k;
    printf("gemm NT %ldx%ldx%ld unmasked: %.3f ms %.2f TFLOP/s\n", n, n, k, base, fl / base / 1e9);
    {
        auto m = mask_bits(ncu, 0, false, true);   // every bit set
        hipStream_t s;
        CHECK(hipExtStreamCreateWithCUMask(&s, uint32_t(m.size() * 32), m.data()));
        double t = gemm_ms(s, n, k, A, B, C, 10);
        printf("gemm on a full CU mask            : %.3f ms %.2f TFLOP/s  rate %.3f\n", t, fl / t / 1e9, base / t);
        CHECK(hipStreamDestroy(s));
    }
    for (int R : Rs)
        for (int strided = 1; strided >= 0; --strided) {
            auto m = mask_bits(ncu, R, strided, true);
            hipStream_t s;
            CHECK(hipExtStreamCreateWithCUMask(&s, uint32_t(m.size() * 32), m.data()));
            double t = gemm_ms(s, n, k, A, B, C, 10);
            printf("gemm on complement of R=%-3d %-9s: %.3f ms %.2f TFLOP/s  rate %.3f  ideal %.3f\n", R,
                   strided ? "strided" : "bits0..R", t, fl / t / 1e9, base / t, double(ncu - R) / ncu);
            CHECK(hipStreamDestroy(s));
        }
    return 0;
}
