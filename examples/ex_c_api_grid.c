/* Multi-process C API example: a p x q grid over a torchrun-style launch
 * (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT), distributed test matrices,
 * an LU solve and its residual, all through the C API. */
#include <math.h>
#include <stdio.h>
#include "slate_amd/c_api.h"

int main(void) {
    if (slate_grid_init(0, 0) != 0) { printf("grid init failed: %s\n", slate_last_error()); return 1; }
    const int64_t n = 400, nrhs = 3, nb = 64;
    slate_Options opts[1] = {{slate_Option_Target, slate_device_available() ? 'D' : 'H', 0.0}};
    slate_Matrix_r64 A = slate_Matrix_create_r64(n, n, nb), A0 = slate_Matrix_create_r64(n, n, nb);
    slate_Matrix_r64 B = slate_Matrix_create_r64(n, nrhs, nb), B0 = slate_Matrix_create_r64(n, nrhs, nb);
    slate_generate_matrix_r64("rands+n", A, 7, -1.0, 1, opts);   /* diagonally dominant */
    slate_generate_matrix_r64("rands", B, 8, -1.0, 1, opts);
    slate_Matrix_insertLocalTiles_r64(A0, (slate_Target)opts[0].ivalue);
    slate_Matrix_insertLocalTiles_r64(B0, (slate_Target)opts[0].ivalue);
    slate_copy_r64(A, A0, 1, opts);
    slate_copy_r64(B, B0, 1, opts);
    int64_t info = slate_lu_solve_r64(A, B, 1, opts);            /* B := X */
    double anorm = slate_norm_r64('1', A0, 1, opts), xnorm = slate_norm_r64('1', B, 1, opts);
    slate_multiply_r64(-1.0, A0, B, 1.0, B0, 1, opts);          /* B0 := B0 - A0 X */
    double res = slate_norm_r64('1', B0, 1, opts) / (n * anorm * xnorm);
    if (slate_grid_rank() == 0)
        printf("slate %s  %d ranks  lu_solve info=%lld residual=%.3e\n", slate_version(), slate_grid_size(),
               (long long)info, res);
    int ok = info == 0 && res < 1e-15;
    slate_Matrix_destroy_r64(A); slate_Matrix_destroy_r64(A0);
    slate_Matrix_destroy_r64(B); slate_Matrix_destroy_r64(B0);
    slate_finalize();
    return ok ? 0 : 1;
}
