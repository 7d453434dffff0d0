// Simplified C++ API (reference include/slate/simplified_api.hh:18-848):
// descriptive names that dispatch on the matrix types to the traditional
// BLAS/LAPACK-named drivers of slate.hh.
#pragma once

#include "slate.hh"

namespace slate {

//------------------------------------------------------------------------------
// Level-3 BLAS

/// C = alpha A B + beta C  (gemm)
template <typename T>
void multiply(T alpha, Matrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C, Options const& opts = {}) {
    gemm(alpha, A, B, beta, C, opts);
}
/// band A (gbmm)
template <typename T>
void multiply(T alpha, BandMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C, Options const& opts = {}) {
    gbmm(alpha, A, B, beta, C, opts);
}
/// Hermitian A on the left / right (hemm)
template <typename T>
void multiply(T alpha, HermitianMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C, Options const& opts = {}) {
    hemm(Side::Left, alpha, A, B, beta, C, opts);
}
template <typename T>
void multiply(T alpha, Matrix<T> const& A, HermitianMatrix<T> const& B, T beta, Matrix<T>& C, Options const& opts = {}) {
    hemm(Side::Right, alpha, B, A, beta, C, opts);
}
/// symmetric A on the left / right (symm)
template <typename T>
void multiply(T alpha, SymmetricMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C, Options const& opts = {}) {
    symm(Side::Left, alpha, A, B, beta, C, opts);
}
template <typename T>
void multiply(T alpha, Matrix<T> const& A, SymmetricMatrix<T> const& B, T beta, Matrix<T>& C, Options const& opts = {}) {
    symm(Side::Right, alpha, B, A, beta, C, opts);
}
/// Hermitian band A on the left / right (hbmm)
template <typename T>
void multiply(T alpha, HermitianBandMatrix<T> const& A, Matrix<T> const& B, T beta, Matrix<T>& C, Options const& opts = {}) {
    hbmm(Side::Left, alpha, A, B, beta, C, opts);
}
template <typename T>
void multiply(T alpha, Matrix<T> const& A, HermitianBandMatrix<T> const& B, T beta, Matrix<T>& C, Options const& opts = {}) {
    hbmm(Side::Right, alpha, B, A, beta, C, opts);
}

/// B = alpha A B or B = alpha B A with triangular A (trmm)
template <typename T>
void triangular_multiply(T alpha, TriangularMatrix<T> const& A, Matrix<T>& B, Options const& opts = {}) {
    trmm(Side::Left, alpha, A, B, opts);
}
template <typename T>
void triangular_multiply(T alpha, Matrix<T>& B, TriangularMatrix<T> const& A, Options const& opts = {}) {
    trmm(Side::Right, alpha, A, B, opts);
}

/// Solve A X = alpha B or X A = alpha B, X overwrites B (trsm, tbsm)
template <typename T>
void triangular_solve(T alpha, TriangularMatrix<T> const& A, Matrix<T>& B, Options const& opts = {}) {
    trsm(Side::Left, alpha, A, B, opts);
}
template <typename T>
void triangular_solve(T alpha, Matrix<T>& B, TriangularMatrix<T> const& A, Options const& opts = {}) {
    trsm(Side::Right, alpha, A, B, opts);
}
template <typename T>
void triangular_solve(T alpha, TriangularBandMatrix<T> const& A, Matrix<T>& B, Options const& opts = {}) {
    tbsm(Side::Left, alpha, A, B, opts);
}
template <typename T>
void triangular_solve(T alpha, Matrix<T>& B, TriangularBandMatrix<T> const& A, Options const& opts = {}) {
    tbsm(Side::Right, alpha, A, B, opts);
}
/// with band LU row interchanges (tbsm with pivots, reference src/tbsmPivots.cc)
template <typename T>
void triangular_solve(T alpha, TriangularBandMatrix<T> const& A, Pivots const& pivots, Matrix<T>& B,
                      Options const& opts = {}) {
    tbsm(Side::Left, alpha, A, pivots, B, opts);
}

/// C = alpha A A^H + beta C (herk) / alpha A A^T + beta C (syrk)
template <typename T>
void rank_k_update(real_type<T> alpha, Matrix<T> const& A, real_type<T> beta, HermitianMatrix<T>& C,
                   Options const& opts = {}) {
    herk(alpha, A, beta, C, opts);
}
template <typename T>
void rank_k_update(T alpha, Matrix<T> const& A, T beta, SymmetricMatrix<T>& C, Options const& opts = {}) {
    syrk(alpha, A, beta, C, opts);
}
/// C = alpha A B^H + conj(alpha) B A^H + beta C (her2k) / syr2k
template <typename T>
void rank_2k_update(T alpha, Matrix<T> const& A, Matrix<T> const& B, real_type<T> beta, HermitianMatrix<T>& C,
                    Options const& opts = {}) {
    her2k(alpha, A, B, beta, C, opts);
}
template <typename T>
void rank_2k_update(T alpha, Matrix<T> const& A, Matrix<T> const& B, T beta, SymmetricMatrix<T>& C, Options const& opts = {}) {
    syr2k(alpha, A, B, beta, C, opts);
}

//------------------------------------------------------------------------------
// LU

template <typename T>
int64_t lu_solve(Matrix<T>& A, Matrix<T>& B, Options const& opts = {}) {
    Pivots pivots;
    return gesv(A, pivots, B, opts);
}
template <typename T>
int64_t lu_solve(BandMatrix<T>& A, Matrix<T>& B, Options const& opts = {}) {
    Pivots pivots;
    return gbsv(A, pivots, B, opts);
}
template <typename T>
int64_t lu_solve_nopiv(Matrix<T>& A, Matrix<T>& B, Options const& opts = {}) {
    return gesv_nopiv(A, B, opts);
}
template <typename T>
int64_t lu_factor(Matrix<T>& A, Pivots& pivots, Options const& opts = {}) {
    return getrf(A, pivots, opts);
}
template <typename T>
int64_t lu_factor(BandMatrix<T>& A, Pivots& pivots, Options const& opts = {}) {
    return gbtrf(A, pivots, opts);
}
template <typename T>
int64_t lu_factor_nopiv(Matrix<T>& A, Options const& opts = {}) {
    return getrf_nopiv(A, opts);
}
template <typename T>
void lu_solve_using_factor(Matrix<T>& A, Pivots& pivots, Matrix<T>& B, Options const& opts = {}) {
    getrs(A, pivots, B, opts);
}
template <typename T>
void lu_solve_using_factor(BandMatrix<T>& A, Pivots& pivots, Matrix<T>& B, Options const& opts = {}) {
    gbtrs(A, pivots, B, opts);
}
template <typename T>
void lu_solve_using_factor_nopiv(Matrix<T>& A, Matrix<T>& B, Options const& opts = {}) {
    getrs_nopiv(A, B, opts);
}
template <typename T>
void lu_inverse_using_factor(Matrix<T>& A, Pivots& pivots, Options const& opts = {}) {
    getri(A, pivots, opts);
}
template <typename T>
void lu_inverse_using_factor_out_of_place(Matrix<T>& A, Pivots& pivots, Matrix<T>& A_inverse,
                                          Options const& opts = {}) {
    getri(A, pivots, A_inverse, opts);
}
template <typename T>
real_type<T> lu_rcondest_using_factor(Norm in_norm, Matrix<T>& A, real_type<T> Anorm, Options const& opts = {}) {
    return gecondest(in_norm, A, Anorm, opts);
}

//------------------------------------------------------------------------------
// Cholesky

template <typename T>
int64_t chol_solve(HermitianMatrix<T>& A, Matrix<T>& B, Options const& opts = {}) {
    return posv(A, B, opts);
}
template <typename T>
int64_t chol_solve(HermitianBandMatrix<T>& A, Matrix<T>& B, Options const& opts = {}) {
    return pbsv(A, B, opts);
}
template <typename T>
int64_t chol_solve(SymmetricMatrix<T>& A, Matrix<T>& B, Options const& opts = {}) {
    static_assert(!is_complex_v<T>, "chol_solve(SymmetricMatrix) is for real types");
    HermitianMatrix<T> H(A.uplo(), A);
    return posv(H, B, opts);
}
template <typename T>
int64_t chol_factor(HermitianMatrix<T>& A, Options const& opts = {}) {
    return potrf(A, opts);
}
template <typename T>
int64_t chol_factor(HermitianBandMatrix<T>& A, Options const& opts = {}) {
    return pbtrf(A, opts);
}
template <typename T>
int64_t chol_factor(SymmetricMatrix<T>& A, Options const& opts = {}) {
    static_assert(!is_complex_v<T>, "chol_factor(SymmetricMatrix) is for real types");
    HermitianMatrix<T> H(A.uplo(), A);
    return potrf(H, opts);
}
template <typename T>
void chol_solve_using_factor(HermitianMatrix<T>& A, Matrix<T>& B, Options const& opts = {}) {
    potrs(A, B, opts);
}
template <typename T>
void chol_solve_using_factor(HermitianBandMatrix<T>& A, Matrix<T>& B, Options const& opts = {}) {
    pbtrs(A, B, opts);
}
template <typename T>
void chol_inverse_using_factor(HermitianMatrix<T>& A, Options const& opts = {}) {
    potri(A, opts);
}
template <typename T>
real_type<T> chol_rcondest_using_factor(Norm in_norm, HermitianMatrix<T>& A, real_type<T> Anorm,
                                        Options const& opts = {}) {
    return pocondest(in_norm, A, Anorm, opts);
}

//------------------------------------------------------------------------------
// Hermitian / symmetric indefinite (Bunch-Kaufman here; LAPACK ipiv)

template <typename T>
int64_t indefinite_solve(HermitianMatrix<T>& A, Matrix<T>& B, Options const& opts = {}) {
    std::vector<int64_t> ipiv;
    return hesv(A, ipiv, B, opts);
}
template <typename T>
int64_t indefinite_solve(SymmetricMatrix<T>& A, Matrix<T>& B, Options const& opts = {}) {
    std::vector<int64_t> ipiv;
    return sysv(A, ipiv, B, opts);
}
template <typename T>
int64_t indefinite_factor(HermitianMatrix<T>& A, std::vector<int64_t>& ipiv, Options const& opts = {}) {
    return hetrf(A, ipiv, opts);
}
template <typename T>
int64_t indefinite_factor(SymmetricMatrix<T>& A, std::vector<int64_t>& ipiv, Options const& opts = {}) {
    return sytrf(A, ipiv, opts);
}
template <typename T>
void indefinite_solve_using_factor(HermitianMatrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B,
                                   Options const& opts = {}) {
    hetrs(A, ipiv, B, opts);
}
template <typename T>
void indefinite_solve_using_factor(SymmetricMatrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B,
                                   Options const& opts = {}) {
    sytrs(A, ipiv, B, opts);
}

//------------------------------------------------------------------------------
// QR / LQ / least squares

template <typename T>
void least_squares_solve(Matrix<T>& A, Matrix<T>& BX, Options const& opts = {}) {
    TriangularFactors<T> T_;
    gels(A, T_, BX, opts);
}
template <typename T>
void qr_factor(Matrix<T>& A, TriangularFactors<T>& T_, Options const& opts = {}) {
    geqrf(A, T_, opts);
}
template <typename T>
void qr_multiply_by_q(Side side, Op op, Matrix<T>& A, TriangularFactors<T>& T_, Matrix<T>& C,
                      Options const& opts = {}) {
    unmqr(side, op, A, T_, C, opts);
}
template <typename T>
void lq_factor(Matrix<T>& A, TriangularFactors<T>& T_, Options const& opts = {}) {
    gelqf(A, T_, opts);
}
template <typename T>
void lq_multiply_by_q(Side side, Op op, Matrix<T>& A, TriangularFactors<T>& T_, Matrix<T>& C,
                      Options const& opts = {}) {
    unmlq(side, op, A, T_, C, opts);
}

//------------------------------------------------------------------------------
// Condition estimate of a triangular matrix

template <typename T>
real_type<T> triangular_rcondest(Norm in_norm, TriangularMatrix<T>& A, Options const& opts = {}) {
    return trcondest(in_norm, A, opts);
}

//------------------------------------------------------------------------------
// Eigenvalues / singular values

template <typename T>
void eig_vals(HermitianMatrix<T>& A, std::vector<real_type<T>>& Lambda, Options const& opts = {}) {
    Matrix<T> Z;
    heev(A, Lambda, Z, opts);
}
template <typename T>
void eig(HermitianMatrix<T>& A, std::vector<real_type<T>>& Lambda, Options const& opts = {}) {
    eig_vals(A, Lambda, opts);
}
template <typename T>
void eig(HermitianMatrix<T>& A, std::vector<real_type<T>>& Lambda, Matrix<T>& Z, Options const& opts = {}) {
    heev(A, Lambda, Z, opts);
}
template <typename T>
void eig_vals(SymmetricMatrix<T>& A, std::vector<real_type<T>>& Lambda, Options const& opts = {}) {
    Matrix<T> Z;
    syev(A, Lambda, Z, opts);
}
template <typename T>
void eig(SymmetricMatrix<T>& A, std::vector<real_type<T>>& Lambda, Options const& opts = {}) {
    eig_vals(A, Lambda, opts);
}
template <typename T>
void eig(SymmetricMatrix<T>& A, std::vector<real_type<T>>& Lambda, Matrix<T>& Z, Options const& opts = {}) {
    syev(A, Lambda, Z, opts);
}
/// generalized A x = lambda B x (itype 1), A B x = lambda x (2), B A x = lambda x (3)
template <typename T>
void eig(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T>& B, std::vector<real_type<T>>& Lambda,
         Matrix<T>& Z, Options const& opts = {}) {
    hegv(itype, A, B, Lambda, Z, opts);
}
template <typename T>
void eig_vals(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T>& B, std::vector<real_type<T>>& Lambda,
              Options const& opts = {}) {
    Matrix<T> Z;
    hegv(itype, A, B, Lambda, Z, opts);
}
template <typename T>
void eig(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T>& B, std::vector<real_type<T>>& Lambda,
         Options const& opts = {}) {
    eig_vals(itype, A, B, Lambda, opts);
}
/// real symmetric generalized problems (sygv)
template <typename T>
void eig(int64_t itype, SymmetricMatrix<T>& A, SymmetricMatrix<T>& B, std::vector<real_type<T>>& Lambda,
         Matrix<T>& Z, Options const& opts = {}) {
    sygv(itype, A, B, Lambda, Z, opts);
}
template <typename T>
void eig_vals(int64_t itype, SymmetricMatrix<T>& A, SymmetricMatrix<T>& B, std::vector<real_type<T>>& Lambda,
              Options const& opts = {}) {
    Matrix<T> Z;
    sygv(itype, A, B, Lambda, Z, opts);
}
template <typename T>
void eig(int64_t itype, SymmetricMatrix<T>& A, SymmetricMatrix<T>& B, std::vector<real_type<T>>& Lambda,
         Options const& opts = {}) {
    eig_vals(itype, A, B, Lambda, opts);
}
template <typename T>
void svd(Matrix<T>& A, std::vector<real_type<T>>& Sigma, Options const& opts = {}) {
    svd_vals(A, Sigma, opts);
}

}  // namespace slate
