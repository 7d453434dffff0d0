// Development check: batched diagonal-block inverse (trtri_blocks) against a
// host forward substitution, per 64 x 64 sub-block, fp32 and fp64.
#include "../kernels/device_common.hh"
#include "../kernels/kernels.hh"
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

using namespace slate_amd::dev;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

template <typename T>
void run(char uplo, char diag, int64_t BS, int64_t nblk) {
    const int64_t n = BS * nblk, lda = n;
    std::vector<T> A(n * n, T(0));
    srand(7);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < n; ++i) {
            bool in = uplo == 'L' ? i >= j : i <= j;
            if (in) A[i + j * lda] = T((rand() / double(RAND_MAX) - 0.5) / std::sqrt(double(BS))) + (i == j ? T(2) : T(0));
        }
    T *dA, *dW, *dwork;
    CHECK(hipMalloc(&dA, n * n * sizeof(T)));
    CHECK(hipMalloc(&dW, nblk * BS * BS * sizeof(T)));
    CHECK(hipMalloc(&dwork, nblk * BS * BS / 2 * sizeof(T)));
    CHECK(hipMemcpy(dA, A.data(), n * n * sizeof(T), hipMemcpyHostToDevice));
    trtri_blocks<T>(uplo, diag, BS, nblk, dA, lda, dW, dwork, 0);
    CHECK(hipDeviceSynchronize());
    std::vector<T> W(nblk * BS * BS);
    CHECK(hipMemcpy(W.data(), dW, W.size() * sizeof(T), hipMemcpyDeviceToHost));
    // check D_t * A_tt == I per 64-block of the product
    for (int64_t t = 0; t < nblk; ++t) {
        const T* Wt = W.data() + t * BS * BS;
        const T* At = A.data() + t * BS * (lda + 1);
        double worst = 0; int64_t wi = -1, wj = -1;
        for (int64_t j = 0; j < BS; ++j)
            for (int64_t i = 0; i < BS; ++i) {
                double s = 0;
                for (int64_t l = 0; l < BS; ++l) {
                    double a = (l == j && diag == 'U') ? 1.0 : double(At[l + j * lda]);
                    bool in = uplo == 'L' ? l >= j : l <= j;
                    if (!in) a = 0;
                    s += double(Wt[i + l * BS]) * a;
                }
                double e = std::fabs(s - (i == j ? 1.0 : 0.0));
                if (!(e <= worst)) { worst = e; wi = i; wj = j; }
            }
        printf("%s uplo=%c diag=%c BS=%ld block %ld: max |D A - I| = %.3e at (%ld, %ld)\n",
               sizeof(T) == 4 ? "float " : "double", uplo, diag, BS, t, worst, wi, wj);
    }
    hipFree(dA); hipFree(dW); hipFree(dwork);
}

int main() {
    for (char uplo : {'L', 'U'}) {
        run<double>(uplo, 'N', 512, 2);
        run<float>(uplo, 'N', 512, 2);
        run<float>(uplo, 'U', 512, 2);
    }
    return 0;
}
