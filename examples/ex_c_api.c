/* C API example (reference examples/c_api/ex*.c capability): LU solve,
 * Cholesky solve, and a GEMM through opaque slate_Matrix handles. */
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include "slate_amd/c_api.h"

int main(void) {
    const int64_t n = 300, nrhs = 2, nb = 64;
    double *A = malloc(sizeof(double) * n * n), *A0 = malloc(sizeof(double) * n * n);
    double *B = malloc(sizeof(double) * n * nrhs), *B0 = malloc(sizeof(double) * n * nrhs);
    srand(7);
    for (int64_t i = 0; i < n * n; ++i) A[i] = A0[i] = (double)rand() / RAND_MAX - 0.5;
    for (int64_t i = 0; i < n; ++i) { A[i + i * n] += n; A0[i + i * n] += n; }
    for (int64_t i = 0; i < n * nrhs; ++i) B[i] = B0[i] = (double)rand() / RAND_MAX;

    slate_Options opts[1] = {{slate_Option_Target, 'H', 0.0}};
    slate_Matrix_r64 As = slate_Matrix_create_fromLAPACK_r64(n, n, A, n, nb);
    slate_Matrix_r64 Bs = slate_Matrix_create_fromLAPACK_r64(n, nrhs, B, n, nb);
    int64_t info = slate_lu_solve_r64(As, Bs, 1, opts);
    slate_Matrix_tileUpdateAllOrigin_r64(Bs);
    double err = 0;
    for (int64_t j = 0; j < nrhs; ++j)
        for (int64_t i = 0; i < n; ++i) {
            double r = -B0[i + j * n];
            for (int64_t k = 0; k < n; ++k) r += A0[i + k * n] * B[k + j * n];
            err = fmax(err, fabs(r));
        }
    printf("slate %s  lu_solve info=%lld max|Ax-b|=%.3e\n", slate_version(), (long long)info, err);
    slate_Matrix_destroy_r64(As);
    slate_Matrix_destroy_r64(Bs);
    free(A); free(A0); free(B); free(B0);
    return (info == 0 && err < 1e-10) ? 0 : 1;
}
