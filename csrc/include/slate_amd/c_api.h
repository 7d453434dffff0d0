/* C API of slate_d35_amd (reference capability: include/slate/c_api/slate.h,
 * types.h, src/c_api/wrappers.cc).  Opaque handles per precision suffix:
 *   r32 = float, r64 = double, c32 = float _Complex, c64 = double _Complex.
 * Matrices live on the process grid installed with slate_grid_init() (one
 * process per GPU; a single process uses the 1x1 grid).  Every driver takes
 * an options array (may be NULL with count 0).  Functions return 0 / info;
 * a C++ exception inside a call is reported through slate_last_error(). */
#ifndef SLATE_AMD_C_API_H
#define SLATE_AMD_C_API_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef char slate_Target;   /* 'H' host, 'D' devices */
typedef char slate_Op;       /* 'N', 'T', 'C' */
typedef char slate_Uplo;     /* 'U', 'L', 'G' */
typedef char slate_Diag;     /* 'N', 'U' */
typedef char slate_Side;     /* 'L', 'R' */
typedef char slate_Norm;     /* '1', 'I', 'F', 'M' */

/* option keys (same numbering as slate::Option) */
enum {
    slate_Option_ChunkSize = 0, slate_Option_Lookahead = 1, slate_Option_BlockSize = 2,
    slate_Option_InnerBlocking = 3, slate_Option_MaxPanelThreads = 4, slate_Option_Tolerance = 5,
    slate_Option_Target = 6, slate_Option_HoldLocalWorkspace = 7, slate_Option_Depth = 8,
    slate_Option_MaxIterations = 9, slate_Option_UseFallbackSolver = 10, slate_Option_PivotThreshold = 11,
    slate_Option_MethodCholQR = 60, slate_Option_MethodEig = 61, slate_Option_MethodGels = 62,
    slate_Option_MethodGemm = 63, slate_Option_MethodHemm = 64, slate_Option_MethodLU = 65,
    slate_Option_MethodTrsm = 66
};

typedef struct {
    int option;
    int64_t ivalue;   /* integer / char-valued options (Target 'D', MethodLU 2, ...) */
    double dvalue;    /* real-valued options (Tolerance, PivotThreshold) */
} slate_Options;

typedef struct slate_Pivots_struct* slate_Pivots;

/* library */
const char* slate_version(void);
const char* slate_last_error(void);
int  slate_device_available(void);
/* install a p x q grid over a single process (p = q = 1), or return the size
 * of the grid that the Python / C++ layer installed */
int  slate_grid_size(void);
/* Create the p x q process grid over all ranks of a torchrun-style launch
 * (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment; RCCL
 * when a GPU is visible, the native TCP transport otherwise).  p = q = 0
 * picks the most square grid.  Returns 0, or -1 (see slate_last_error). */
int  slate_grid_init(int p, int q);
/* This process's rank in the grid. */
int  slate_grid_rank(void);
/* Barrier and tear down the grid (MPI_Finalize analog). */
void slate_finalize(void);

slate_Pivots slate_Pivots_create(void);
void    slate_Pivots_destroy(slate_Pivots p);
int64_t slate_Pivots_size(slate_Pivots p);

#define SLATE_C_API_DECLARE(X, scalar_t, real_t)                                                          \
typedef struct slate_Matrix_##X##_struct* slate_Matrix_##X;                                               \
typedef struct slate_TriangularFactors_##X##_struct* slate_TriangularFactors_##X;                         \
slate_Matrix_##X slate_Matrix_create_##X(int64_t m, int64_t n, int64_t nb);                               \
slate_Matrix_##X slate_Matrix_create_fromLAPACK_##X(int64_t m, int64_t n, scalar_t* A, int64_t lda,       \
                                                    int64_t nb);                                          \
slate_Matrix_##X slate_Matrix_create_fromScaLAPACK_##X(int64_t m, int64_t n, scalar_t* A, int64_t lld,    \
                                                       int64_t mb, int64_t nb);                           \
void    slate_Matrix_destroy_##X(slate_Matrix_##X A);                                                     \
void    slate_Matrix_insertLocalTiles_##X(slate_Matrix_##X A, slate_Target target);                      \
void    slate_Matrix_tileUpdateAllOrigin_##X(slate_Matrix_##X A);                                        \
int64_t slate_Matrix_m_##X(slate_Matrix_##X A);                                                           \
int64_t slate_Matrix_n_##X(slate_Matrix_##X A);                                                           \
int64_t slate_Matrix_mt_##X(slate_Matrix_##X A);                                                          \
int64_t slate_Matrix_nt_##X(slate_Matrix_##X A);                                                          \
slate_Matrix_##X slate_Matrix_transpose_##X(slate_Matrix_##X A);                                          \
slate_Matrix_##X slate_Matrix_conj_transpose_##X(slate_Matrix_##X A);                                     \
slate_Matrix_##X slate_Matrix_sub_##X(slate_Matrix_##X A, int64_t i1, int64_t i2, int64_t j1, int64_t j2); \
/* copy the matrix's local data to / from a LAPACK array (1 process) */                                   \
int  slate_Matrix_get_##X(slate_Matrix_##X A, scalar_t* out, int64_t ld);                                 \
int  slate_Matrix_set_##X(slate_Matrix_##X A, scalar_t const* in, int64_t ld);                            \
slate_TriangularFactors_##X slate_TriangularFactors_create_##X(void);                                     \
void slate_TriangularFactors_destroy_##X(slate_TriangularFactors_##X T);                                  \
/* level 3 BLAS (uplo / diag select the triangle / diagonal of A where relevant) */                       \
int slate_multiply_##X(scalar_t alpha, slate_Matrix_##X A, slate_Matrix_##X B, scalar_t beta,             \
                       slate_Matrix_##X C, int nopts, slate_Options const* opts);                         \
int slate_hermitian_multiply_##X(slate_Side side, scalar_t alpha, slate_Uplo uplo, slate_Matrix_##X A,    \
                                 slate_Matrix_##X B, scalar_t beta, slate_Matrix_##X C, int nopts,        \
                                 slate_Options const* opts);                                              \
int slate_rank_k_update_##X(real_t alpha, slate_Matrix_##X A, real_t beta, slate_Uplo uplo,               \
                            slate_Matrix_##X C, int nopts, slate_Options const* opts);                    \
int slate_rank_2k_update_##X(scalar_t alpha, slate_Matrix_##X A, slate_Matrix_##X B, real_t beta,         \
                             slate_Uplo uplo, slate_Matrix_##X C, int nopts, slate_Options const* opts);  \
int slate_triangular_multiply_##X(slate_Side side, scalar_t alpha, slate_Uplo uplo, slate_Diag diag,      \
                                  slate_Matrix_##X A, slate_Matrix_##X B, int nopts,                      \
                                  slate_Options const* opts);                                             \
int slate_triangular_solve_##X(slate_Side side, scalar_t alpha, slate_Uplo uplo, slate_Diag diag,         \
                               slate_Matrix_##X A, slate_Matrix_##X B, int nopts,                         \
                               slate_Options const* opts);                                                \
/* norms */                                                                                                \
real_t slate_norm_##X(slate_Norm norm, slate_Matrix_##X A, int nopts, slate_Options const* opts);         \
/* LU */                                                                                                   \
int64_t slate_lu_factor_##X(slate_Matrix_##X A, slate_Pivots pivots, int nopts, slate_Options const* opts); \
int64_t slate_lu_solve_##X(slate_Matrix_##X A, slate_Matrix_##X B, int nopts, slate_Options const* opts); \
int slate_lu_solve_using_factor_##X(slate_Matrix_##X A, slate_Pivots pivots, slate_Matrix_##X B,          \
                                    int nopts, slate_Options const* opts);                                \
int64_t slate_lu_inverse_using_factor_##X(slate_Matrix_##X A, slate_Pivots pivots, int nopts,             \
                                          slate_Options const* opts);                                     \
real_t slate_lu_rcondest_using_factor_##X(slate_Norm norm, slate_Matrix_##X A, real_t anorm, int nopts,   \
                                          slate_Options const* opts);                                     \
int64_t slate_lu_factor_nopiv_##X(slate_Matrix_##X A, int nopts, slate_Options const* opts);             \
/* Cholesky (A's uplo triangle holds the Hermitian matrix / factor) */                                    \
int64_t slate_chol_factor_##X(slate_Uplo uplo, slate_Matrix_##X A, int nopts, slate_Options const* opts); \
int64_t slate_chol_solve_##X(slate_Uplo uplo, slate_Matrix_##X A, slate_Matrix_##X B, int nopts,          \
                             slate_Options const* opts);                                                  \
int slate_chol_solve_using_factor_##X(slate_Uplo uplo, slate_Matrix_##X A, slate_Matrix_##X B, int nopts, \
                                      slate_Options const* opts);                                         \
int64_t slate_chol_inverse_using_factor_##X(slate_Uplo uplo, slate_Matrix_##X A, int nopts,               \
                                            slate_Options const* opts);                                   \
real_t slate_chol_rcondest_using_factor_##X(slate_Norm norm, slate_Uplo uplo, slate_Matrix_##X A,         \
                                            real_t anorm, int nopts, slate_Options const* opts);          \
/* Hermitian indefinite */                                                                                 \
int64_t slate_indefinite_solve_##X(slate_Uplo uplo, slate_Matrix_##X A, slate_Matrix_##X B, int nopts,    \
                                   slate_Options const* opts);                                            \
/* QR / LQ / least squares */                                                                              \
int slate_qr_factor_##X(slate_Matrix_##X A, slate_TriangularFactors_##X T, int nopts,                     \
                        slate_Options const* opts);                                                       \
int slate_qr_multiply_by_q_##X(slate_Side side, slate_Op op, slate_Matrix_##X A,                          \
                               slate_TriangularFactors_##X T, slate_Matrix_##X C, int nopts,              \
                               slate_Options const* opts);                                                \
int slate_lq_factor_##X(slate_Matrix_##X A, slate_TriangularFactors_##X T, int nopts,                     \
                        slate_Options const* opts);                                                       \
int slate_lq_multiply_by_q_##X(slate_Side side, slate_Op op, slate_Matrix_##X A,                          \
                               slate_TriangularFactors_##X T, slate_Matrix_##X C, int nopts,              \
                               slate_Options const* opts);                                                \
int slate_least_squares_solve_##X(slate_Matrix_##X A, slate_Matrix_##X BX, int nopts,                     \
                                  slate_Options const* opts);                                             \
/* eigenvalues / SVD: Lambda (n) and Sigma (min(m,n)) are real arrays; Z, U, VT may be NULL */            \
int slate_hermitian_eig_##X(slate_Uplo uplo, slate_Matrix_##X A, real_t* Lambda, slate_Matrix_##X Z,      \
                            int nopts, slate_Options const* opts);                                        \
int slate_svd_##X(slate_Matrix_##X A, real_t* Sigma, slate_Matrix_##X U, slate_Matrix_##X VT, int nopts,  \
                  slate_Options const* opts);                                                             \
/* auxiliary */                                                                                            \
int slate_copy_##X(slate_Matrix_##X A, slate_Matrix_##X B, int nopts, slate_Options const* opts);         \
int slate_add_##X(scalar_t alpha, slate_Matrix_##X A, scalar_t beta, slate_Matrix_##X B, int nopts,       \
                  slate_Options const* opts);                                                             \
int slate_scale_##X(real_t numer, real_t denom, slate_Matrix_##X A, int nopts, slate_Options const* opts); \
int slate_set_##X(scalar_t offdiag, scalar_t diag, slate_Matrix_##X A, int nopts, slate_Options const* opts); \
/* test matrices (matgen kinds: "rand", "rands", "randn", "spd", "rands+n", ... ; shift < 0: default) */   \
int slate_generate_matrix_##X(const char* kind, slate_Matrix_##X A, uint64_t seed, double shift,           \
                              int nopts, slate_Options const* opts);

#ifdef __cplusplus
#define SLATE_C32 _slate_c32
#define SLATE_C64 _slate_c64
typedef struct { float re, im; } _slate_c32;
typedef struct { double re, im; } _slate_c64;
#else
#include <complex.h>
#define SLATE_C32 float _Complex
#define SLATE_C64 double _Complex
#endif

SLATE_C_API_DECLARE(r32, float, float)
SLATE_C_API_DECLARE(r64, double, double)
SLATE_C_API_DECLARE(c32, SLATE_C32, float)
SLATE_C_API_DECLARE(c64, SLATE_C64, double)

/* mixed precision (fp32 factorization + fp64 refinement) */
int64_t slate_lu_solve_mixed_r64(slate_Matrix_r64 A, slate_Matrix_r64 B, slate_Matrix_r64 X, int* iter,
                                 int nopts, slate_Options const* opts);
int64_t slate_chol_solve_mixed_r64(slate_Uplo uplo, slate_Matrix_r64 A, slate_Matrix_r64 B, slate_Matrix_r64 X,
                                   int* iter, int nopts, slate_Options const* opts);

#ifdef __cplusplus
}
#endif

#endif /* SLATE_AMD_C_API_H */
