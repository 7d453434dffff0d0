// Public C++ API (reference include/slate/slate.hh:43-1410).
//
// Traditional BLAS/LAPACK-named drivers taking distributed matrices and an
// Options map.  Option::Target selects Host (C++/OpenMP tile kernels) or
// Devices (gfx950 HIP kernels on this process's GPU).  Every driver is
// collective over the matrices' process grid.
#pragma once

#include "enums.hh"
#include "types.hh"
#include "exception.hh"
#include "util.hh"
#include "device.hh"
#include "comm.hh"
#include "grid.hh"
#include "matrix.hh"
#include "inproc.hh"
#include "func.hh"
#include "method.hh"
#include "matgen.hh"
#include "init.hh"
#include "eig_host.hh"
#include "debug.hh"

#include <vector>

namespace slate {

/// T factors of a QR/LQ factorization: T[0] holds one nb x nb block per
/// panel (block column k -> columns [k*nb, (k+1)*nb) of an nb x n matrix
/// replicated on the panel's process column).
template <typename T>
using TriangularFactors = std::vector<Matrix<T>>;

//------------------------------------------------------------------------------
// Level-3 BLAS
template <typename T>
void gemm(T alpha, Matrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C, Options const& opts = {});
template <typename T>
void gemmA(T alpha, Matrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C, Options const& opts = {});
template <typename T>
void gemmC(T alpha, Matrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C, Options const& opts = {});

template <typename T>
void hemm(Side side, T alpha, HermitianMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C,
          Options const& opts = {});
template <typename T>
void symm(Side side, T alpha, SymmetricMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C,
          Options const& opts = {});
template <typename T>
void herk(real_type<T> alpha, Matrix<T> const& A, real_type<T> beta, HermitianMatrix<T>& C, Options const& opts = {});
template <typename T>
void syrk(T alpha, Matrix<T> const& A, T beta, SymmetricMatrix<T>& C, Options const& opts = {});
template <typename T>
void her2k(T alpha, Matrix<T> const& A, Matrix<T> const& B, real_type<T> beta, HermitianMatrix<T>& C,
           Options const& opts = {});
template <typename T>
void syr2k(T alpha, Matrix<T> const& A, Matrix<T> const& B, T beta, SymmetricMatrix<T>& C, Options const& opts = {});
template <typename T>
void trmm(Side side, T alpha, TriangularMatrix<T> const& A, Matrix<T>& B, Options const& opts = {});
template <typename T>
void trsm(Side side, T alpha, TriangularMatrix<T> const& A, Matrix<T>& B, Options const& opts = {});

/// Method-specific entry points (reference slate.hh hemmA / hemmC / trsmA /
/// trsmB): the generic driver with the method option fixed.
template <typename T>
inline void hemmA(Side side, T alpha, HermitianMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C,
                  Options const& opts = {}) {
    Options o = opts;
    o[Option::MethodHemm] = int64_t(MethodHemm::HemmA);
    hemm(side, alpha, A, B, beta, C, o);
}
template <typename T>
inline void hemmC(Side side, T alpha, HermitianMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C,
                  Options const& opts = {}) {
    Options o = opts;
    o[Option::MethodHemm] = int64_t(MethodHemm::HemmC);
    hemm(side, alpha, A, B, beta, C, o);
}
template <typename T>
inline void trsmA(Side side, T alpha, TriangularMatrix<T> const& A, Matrix<T>& B, Options const& opts = {}) {
    Options o = opts;
    o[Option::MethodTrsm] = int64_t(MethodTrsm::TrsmA);
    trsm(side, alpha, A, B, o);
}
template <typename T>
inline void trsmB(Side side, T alpha, TriangularMatrix<T> const& A, Matrix<T>& B, Options const& opts = {}) {
    Options o = opts;
    o[Option::MethodTrsm] = int64_t(MethodTrsm::TrsmB);
    trsm(side, alpha, A, B, o);
}

//------------------------------------------------------------------------------
// Auxiliary
template <typename T>
void add(T alpha, Matrix<T> const& A, T beta, Matrix<T>& B, Options const& opts = {});
template <typename T>
void add(T alpha, BaseTrapezoidMatrix<T> const& A, T beta, BaseTrapezoidMatrix<T>& B, Options const& opts = {});
template <typename Ts, typename Td>
void copy(BaseMatrix<Ts> const& A, BaseMatrix<Td>& B, Options const& opts = {});
template <typename T>
void scale(real_type<T> numer, real_type<T> denom, BaseMatrix<T>& A, Options const& opts = {});
template <typename T>
void scale_row_col(Equed equed, std::vector<real_type<T>> const& R, std::vector<real_type<T>> const& C,
                   Matrix<T>& A, Options const& opts = {});
template <typename T>
void set(T offdiag, T diag, BaseMatrix<T>& A, Options const& opts = {});
/// Set each element via a lambda of global indices (reference set_lambdas.cc).
template <typename T>
void set(std::function<T(int64_t, int64_t)> const& value, BaseMatrix<T>& A, Options const& opts = {});
/// Gather the whole matrix to every rank's host array (ld = m).
template <typename T>
void gather(BaseMatrix<T> const& A, std::vector<T>& full, Options const& opts = {});
/// B = A with any source/target distributions (reference redistribute.cc).
template <typename T>
void redistribute(Matrix<T> const& A, Matrix<T>& B, Options const& opts = {});

//------------------------------------------------------------------------------
// Norms (reference norm.cc, colNorms.cc)
template <typename T>
real_type<T> norm(Norm norm, BaseMatrix<T> const& A, Options const& opts = {});
template <typename T>
void colNorms(Norm norm, Matrix<T> const& A, real_type<T>* values, Options const& opts = {});

//------------------------------------------------------------------------------
// Cholesky
template <typename T>
int64_t potrf(HermitianMatrix<T>& A, Options const& opts = {});
template <typename T>
void potrs(HermitianMatrix<T> const& A, Matrix<T>& B, Options const& opts = {});
template <typename T>
int64_t posv(HermitianMatrix<T>& A, Matrix<T>& B, Options const& opts = {});
template <typename T>
int64_t potri(HermitianMatrix<T>& A, Options const& opts = {});
template <typename T>
int64_t posv_mixed(HermitianMatrix<T>& A, Matrix<T>& B, Matrix<T>& X, int& iter, Options const& opts = {});
template <typename T>
[[deprecated("Use posv_mixed")]] inline int64_t posvMixed(HermitianMatrix<T>& A, Matrix<T>& B, Matrix<T>& X, int& iter,
                                                         Options const& opts = {}) {
    return posv_mixed(A, B, X, iter, opts);
}
template <typename T>
int64_t posv_mixed_gmres(HermitianMatrix<T>& A, Matrix<T>& B, Matrix<T>& X, int& iter, Options const& opts = {});
template <typename T>
real_type<T> pocondest(Norm in_norm, HermitianMatrix<T>& A, real_type<T> Anorm, Options const& opts = {});

//------------------------------------------------------------------------------
// LU
template <typename T>
int64_t getrf(Matrix<T>& A, Pivots& pivots, Options const& opts = {});
template <typename T>
int64_t getrf_nopiv(Matrix<T>& A, Options const& opts = {});
template <typename T>
int64_t getrf_tntpiv(Matrix<T>& A, Pivots& pivots, Options const& opts = {});
/// Exact LU row-exchange counters of this process (diagnostics / tests):
/// elements sent and rows sent (summed over column ranges) since the reset.
void lu_rowx_stats(int64_t& elems, int64_t& rows);
void lu_rowx_reset();
template <typename T>
void getrs(Matrix<T> const& A, Pivots const& pivots, Matrix<T>& B, Options const& opts = {});
template <typename T>
void getrs_nopiv(Matrix<T> const& A, Matrix<T>& B, Options const& opts = {});
template <typename T>
int64_t gesv(Matrix<T>& A, Pivots& pivots, Matrix<T>& B, Options const& opts = {});
template <typename T>
int64_t gesv_nopiv(Matrix<T>& A, Matrix<T>& B, Options const& opts = {});
template <typename T>
int64_t gesv_mixed(Matrix<T>& A, Pivots& pivots, Matrix<T>& B, Matrix<T>& X, int& iter, Options const& opts = {});
/// (reference's older camel-case name)
template <typename T>
[[deprecated("Use gesv_mixed")]] inline int64_t gesvMixed(Matrix<T>& A, Pivots& pivots, Matrix<T>& B, Matrix<T>& X,
                                                         int& iter, Options const& opts = {}) {
    return gesv_mixed(A, pivots, B, X, iter, opts);
}
template <typename T>
int64_t gesv_mixed_gmres(Matrix<T>& A, Pivots& pivots, Matrix<T>& B, Matrix<T>& X, int& iter,
                         Options const& opts = {});
template <typename T>
int64_t getri(Matrix<T>& A, Pivots const& pivots, Options const& opts = {});
template <typename T>
real_type<T> gecondest(Norm in_norm, Matrix<T>& A, real_type<T> Anorm, Options const& opts = {});
template <typename T>
int64_t trtri(TriangularMatrix<T>& A, Options const& opts = {});
template <typename T>
void trtrm(TriangularMatrix<T>& A, Options const& opts = {});
template <typename T>
real_type<T> trcondest(Norm in_norm, TriangularMatrix<T>& A, Options const& opts = {});

//------------------------------------------------------------------------------
// QR / LQ / least squares
template <typename T>
void geqrf(Matrix<T>& A, TriangularFactors<T>& T_, Options const& opts = {});
template <typename T>
void unmqr(Side side, Op op, Matrix<T> const& A, TriangularFactors<T> const& T_, Matrix<T>& C,
           Options const& opts = {});
template <typename T>
void gelqf(Matrix<T>& A, TriangularFactors<T>& T_, Options const& opts = {});
template <typename T>
void unmlq(Side side, Op op, Matrix<T> const& A, TriangularFactors<T> const& T_, Matrix<T>& C,
           Options const& opts = {});
template <typename T>
void gels(Matrix<T>& A, TriangularFactors<T>& T_, Matrix<T>& BX, Options const& opts = {});
template <typename T>
int64_t cholqr(Matrix<T>& A, Matrix<T>& R, Options const& opts = {});

//------------------------------------------------------------------------------
// Eigenvalues / SVD (host-centric, reference heev.cc / svd.cc)
template <typename T>
void heev(HermitianMatrix<T>& A, std::vector<real_type<T>>& Lambda, Matrix<T>& Z, Options const& opts = {});
template <typename T>
void svd(Matrix<T>& A, std::vector<real_type<T>>& Sigma, Matrix<T>& U, Matrix<T>& VT, Options const& opts = {});
/// Stage 1 of heev: Hermitian (dense general storage) -> band of width nb.
template <typename T>
void he2hb(Matrix<T>& A, std::vector<TriangularFactors<T>>& Ts, Options const& opts = {});
/// Stage 1 of svd: general (m >= n) -> upper band of width nb.
template <typename T>
void ge2tb(Matrix<T>& A, std::vector<TriangularFactors<T>>& TU, std::vector<TriangularFactors<T>>& TV,
           Options const& opts = {});
template <typename T>
void hegst(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T> const& B, Options const& opts = {});
template <typename T>
void hegv(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T>& B, std::vector<real_type<T>>& Lambda,
          Matrix<T>& Z, Options const& opts = {});

//------------------------------------------------------------------------------
// Band (reference gbtrf.cc, gbtrs.cc, gbsv.cc, pbtrf.cc, pbtrs.cc, pbsv.cc,
// gbmm.cc, hbmm.cc, tbsm.cc)
template <typename T>
int64_t gbtrf(BandMatrix<T>& A, Pivots& pivots, Options const& opts = {});
template <typename T>
void gbtrs(BandMatrix<T> const& A, Pivots const& pivots, Matrix<T>& B, Options const& opts = {});
template <typename T>
int64_t gbsv(BandMatrix<T>& A, Pivots& pivots, Matrix<T>& B, Options const& opts = {});
template <typename T>
int64_t pbtrf(HermitianBandMatrix<T>& A, Options const& opts = {});
template <typename T>
void pbtrs(HermitianBandMatrix<T> const& A, Matrix<T>& B, Options const& opts = {});
template <typename T>
int64_t pbsv(HermitianBandMatrix<T>& A, Matrix<T>& B, Options const& opts = {});
template <typename T>
void gbmm(T alpha, BandMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C, Options const& opts = {});
template <typename T>
void hbmm(Side side, T alpha, HermitianBandMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C,
          Options const& opts = {});
template <typename T>
void tbsm(Side side, T alpha, TriangularBandMatrix<T> const& A, Matrix<T>& B, Options const& opts = {});
/// tbsm with gbtrf's row interchanges (reference slate.hh:305-310,
/// src/tbsmPivots.cc): the interchanges of tile k are applied to
/// B(k:mt-1, :) before tile k's solve on a forward sweep (op(A) lower, the L
/// of gbtrf) or after it on a backward sweep (op(A) upper); empty pivots =
/// plain tbsm.
template <typename T>
void tbsm(Side side, T alpha, TriangularBandMatrix<T> const& A, Pivots const& pivots, Matrix<T>& B,
          Options const& opts = {});

//------------------------------------------------------------------------------
// Hermitian indefinite (reference hetrf.cc, hetrs.cc, hesv.cc); LAPACK ipiv.
template <typename T>
int64_t hetrf(HermitianMatrix<T>& A, std::vector<int64_t>& ipiv, Options const& opts = {});
template <typename T>
void hetrs(HermitianMatrix<T> const& A, std::vector<int64_t> const& ipiv, Matrix<T>& B, Options const& opts = {});
template <typename T>
int64_t hesv(HermitianMatrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B, Options const& opts = {});
// Aasen (reference hetrf.cc signatures): P A P^T = L T L^H, T band (kl = ku = nb)
template <typename T>
int64_t hetrf(HermitianMatrix<T>& A, Pivots& pivots, BandMatrix<T>& T_, Pivots& pivots2, Matrix<T>& H,
              Options const& opts = {});
template <typename T>
void hetrs(HermitianMatrix<T>& A, Pivots& pivots, BandMatrix<T>& T_, Pivots& pivots2, Matrix<T>& B,
           Options const& opts = {});
template <typename T>
int64_t hesv(HermitianMatrix<T>& A, Pivots& pivots, BandMatrix<T>& T_, Pivots& pivots2, Matrix<T>& H, Matrix<T>& B,
             Options const& opts = {});

/// op(A) X = B with getrf factors (op = NoTrans, Trans, ConjTrans).
template <typename T>
void getrs(Op trans, Matrix<T> const& A, Pivots const& pivots, Matrix<T>& B, Options const& opts = {});
/// Out-of-place inverse from getrf factors (reference getriOOP.cc).
template <typename T>
int64_t getri(Matrix<T>& A, Pivots const& pivots, Matrix<T>& B, Options const& opts);
/// Random butterfly transform A := U^T A V and the RBT solver (gerbt.cc, gesv_rbt.cc).
template <typename T>
void gerbt(Matrix<T>& A, int depth, uint64_t seed_u, uint64_t seed_v, Options const& opts = {});
template <typename T>
int64_t gesv_rbt(Matrix<T>& A, Matrix<T>& B, Matrix<T>& X, int& iter, Options const& opts = {});

//------------------------------------------------------------------------------
// Two-stage reduction building blocks (reference slate.hh:1050-1334).
/// Householder reflectors of a bulge-chasing stage (hb2st / tb2bd) plus the
/// diagonal phase that makes the condensed form real; replicated on every
/// rank (the reference keeps them in a distributed Matrix V).
template <typename T>
struct BandReflectors {
    host::Reflectors<T> Q;
    std::vector<T> phase;
};

/// Band Hermitian -> real symmetric tridiagonal (D, E); A = Q T Q^H with
/// Q = V.Q diag(V.phase).
template <typename T>
void hb2st(HermitianBandMatrix<T>& A, std::vector<real_type<T>>& D, std::vector<real_type<T>>& E,
           BandReflectors<T>& V, Options const& opts = {});
/// C = op(Q) C (Side::Left) or C op(Q) (Side::Right) with Q from hb2st.
template <typename T>
void unmtr_hb2st(Side side, Op op, BandReflectors<T> const& V, Matrix<T>& C, Options const& opts = {});
/// C = op(Q1) C / C op(Q1) with Q1 the he2hb reflectors (stored below the band of A).
template <typename T>
void unmtr_he2hb(Side side, Op op, Matrix<T>& A, std::vector<TriangularFactors<T>>& Ts, Matrix<T>& C,
                 Options const& opts = {});
/// Upper triangular band -> real upper bidiagonal: A = U B V^H.
template <typename T>
void tb2bd(TriangularBandMatrix<T>& A, std::vector<real_type<T>>& D, std::vector<real_type<T>>& E,
           BandReflectors<T>& U, BandReflectors<T>& V, Options const& opts = {});
/// Apply the tb2bd reflectors U or V: C = op(Q) C or C op(Q).
template <typename T>
void unmbr_tb2bd(Side side, Op op, BandReflectors<T> const& V, Matrix<T>& C, Options const& opts = {});
/// Apply the ge2tb reflectors: Side::Left with the QR factors TU (C = op(U1) C),
/// Side::Right with the LQ factors TV (C = C op(V1^H)).
template <typename T>
void unmbr_ge2tb(Side side, Op op, Matrix<T>& A, std::vector<TriangularFactors<T>>& Ts, Matrix<T>& C,
                 Options const& opts = {});

/// Tridiagonal eigenvalues only (root-free QL).
template <typename R>
void sterf(std::vector<R>& D, std::vector<R>& E, Options const& opts = {});
/// Tridiagonal QL/QR; with jobz = Vec, Z := Z * (eigenvectors).
template <typename T>
void steqr2(Job jobz, std::vector<real_type<T>>& D, std::vector<real_type<T>>& E, Matrix<T>& Z,
            Options const& opts = {});
/// Tridiagonal divide and conquer: eigenvalues ascending in D, vectors in Q.
template <typename R>
void stedc(std::vector<R>& D, std::vector<R>& E, Matrix<R>& Q, Options const& opts = {});
/// D&C stages (reference stedc_solve.cc, stedc_z_vector.cc, stedc_sort.cc,
/// stedc_deflate.cc, stedc_secular.cc, stedc_merge.cc).
template <typename R>
void stedc_solve(std::vector<R>& D, std::vector<R>& E, Matrix<R>& Q, Options const& opts = {});
template <typename R>
void stedc_z_vector(Matrix<R>& Q, int64_t n1, R sgn, std::vector<R>& z, Options const& opts = {});
template <typename R>
void stedc_sort(std::vector<R>& D, std::vector<R>& z, Matrix<R>& Q, Matrix<R>& Qout, std::vector<int64_t>& perm,
                Options const& opts = {});
template <typename R>
int64_t stedc_deflate(R rho, std::vector<R>& D, std::vector<R>& z, Matrix<R>& Q, std::vector<char>& deflated,
                      Options const& opts = {});
template <typename R>
void stedc_secular(R rho, std::vector<R> const& D, std::vector<R> const& z, std::vector<R>& Lambda, Matrix<R>& U,
                   Options const& opts = {});
template <typename R>
void stedc_merge(Matrix<R>& Q, Matrix<R>& U, Matrix<R>& Qout, Options const& opts = {});
/// Bidiagonal SVD: D descending singular values; U := U Ub, VT := Vb^H VT.
template <typename T>
void bdsqr(Job jobu, Job jobvt, std::vector<real_type<T>>& D, std::vector<real_type<T>>& E, Matrix<T>& U,
           Matrix<T>& VT, Options const& opts = {});

//------------------------------------------------------------------------------
// Real-symmetric aliases (real types only) and compatibility names.
template <typename T>
void syev(SymmetricMatrix<T>& A, std::vector<real_type<T>>& Lambda, Matrix<T>& Z, Options const& opts = {});
template <typename T>
void sygst(int64_t itype, SymmetricMatrix<T>& A, SymmetricMatrix<T> const& B, Options const& opts = {});
template <typename T>
void sygv(int64_t itype, SymmetricMatrix<T>& A, SymmetricMatrix<T>& B, std::vector<real_type<T>>& Lambda,
          Matrix<T>& Z, Options const& opts = {});
template <typename T>
int64_t sytrf(SymmetricMatrix<T>& A, std::vector<int64_t>& ipiv, Options const& opts = {});
template <typename T>
void sytrs(SymmetricMatrix<T> const& A, std::vector<int64_t> const& ipiv, Matrix<T>& B, Options const& opts = {});
template <typename T>
int64_t sysv(SymmetricMatrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B, Options const& opts = {});
template <typename T>
void svd_vals(Matrix<T>& A, std::vector<real_type<T>>& Sigma, Options const& opts = {});
template <typename T>
void gesvd(Matrix<T>& A, std::vector<real_type<T>>& Sigma, Matrix<T>& U, Matrix<T>& VT, Options const& opts = {});
template <typename T>
void gels_qr(Matrix<T>& A, TriangularFactors<T>& T_, Matrix<T>& BX, Options const& opts = {});
/// Least squares via CholeskyQR (m >= n): A := Q, R upper n x n.
template <typename T>
void gels_cholqr(Matrix<T>& A, Matrix<T>& R, Matrix<T>& BX, Options const& opts = {});

//------------------------------------------------------------------------------
// Printing (reference include/slate/print.hh).  Collective; rank 0 prints a
// MATLAB-style `label = [ ... ];` block.  Options PrintVerbose (0-4, default
// 2 = edges), PrintEdgeItems (16), PrintWidth (10), PrintPrecision (4).
template <typename T>
void print(const char* label, BaseMatrix<T> const& A, Options const& opts = {});
/// Vector x[0:n:incx] (rank 0 only).
template <typename T>
void print(const char* label, int64_t n, T const* x, int64_t incx = 1, Options const& opts = {});
/// What print() writes on rank 0, as a string (empty elsewhere).
template <typename T>
std::string print_to_string(const char* label, BaseMatrix<T> const& A, Options const& opts = {});
template <typename R>
int snprintf_value(char* buf, size_t len, int width, int precision, R value);

/// Wait for all device work of this process (drivers already synchronize).
void sync();

}  // namespace slate

#include "simplified_api.hh"
