// Host (CPU, OpenMP) stages of the two-stage eigenvalue / SVD reductions.
//
// Reference: hb2st.cc (bulge chasing on one node with OpenMP tasks),
// tb2bd.cc, sterf.cc / steqr2.cc / stedc*.cc (tridiagonal eigensolvers),
// bdsqr.cc (bidiagonal SVD through LAPACK++).  There is no vendor LAPACK in
// this stack, so the small dense kernels are written here:
//   * hb2st  Householder bulge chasing, band Hermitian -> real tridiagonal
//   * tb2bd  Householder bulge chasing, upper band -> real upper bidiagonal
//   * steqr  implicit QL with Wilkinson shifts (EISPACK tql2 formulation);
//            rotations of one sweep are applied to Z rows in parallel
//   * stedc  Cuppen divide and conquer with deflation and Gu-Eisenstat
//            eigenvectors; the merge products use the blocked host gemm
//   * bdsqr  Golub-Reinsch implicit-shift QR on the bidiagonal
// The reflectors of hb2st / tb2bd are kept (Reflectors) and applied to the
// eigen/singular vectors afterwards, in reverse order (reference
// unmtr_hb2st.cc / unmbr_tb2bd).
#pragma once

#include "types.hh"

#include <cstdint>
#include <vector>

namespace slate {
namespace host {

/// A sequence of Householder reflectors H_k = I - tau_k v_k v_k^H acting on
/// rows [off_k, off_k + len_k).  Q = H_0 H_1 ... H_{K-1}.
template <typename T>
struct Reflectors {
    std::vector<int64_t> off, len, voff;
    std::vector<int64_t> tag;   // producer's label (hb2st: the sweep), -1 if none
    std::vector<T> tau, v;
    void push(int64_t o, int64_t l, T t, T const* vec, int64_t tg = -1) {
        off.push_back(o); len.push_back(l); voff.push_back(int64_t(v.size())); tau.push_back(t);
        tag.push_back(tg);
        v.insert(v.end(), vec, vec + l);
    }
    size_t size() const { return tau.size(); }
    /// C = Q C (trans = false) or Q^H C (trans = true); C is n_rows x ncols.
    void apply_left(bool trans, int64_t ncols, T* C, int64_t ldc) const;
};

/// Hermitian band (lower, bandwidth kd) to real symmetric tridiagonal (d, e).
/// A is addressed as A[i + j lda] for |i - j| <= 2 kd only, so either dense
/// n x n storage or general band storage with kl = ku = 2 kd works (through
/// the skew A = ab + 2 kd, lda = ldab - 1).  Reflectors (tagged with their
/// sweep) and the diagonal phase (A = Q diag(phase) T diag(phase)^H Q^H) are
/// returned for the back-transform.
template <typename T>
void hb2st(int64_t n, int64_t kd, T* A, int64_t lda, std::vector<real_type<T>>& d, std::vector<real_type<T>>& e,
           Reflectors<T>& Q, std::vector<T>& phase);

/// Upper band (bandwidth kd, dense m x n storage, m >= n) to real upper
/// bidiagonal: A = U B V^H with U = QU diag(pu), V = QV diag(pv).
template <typename T>
void tb2bd(int64_t m, int64_t n, int64_t kd, T* A, int64_t lda, std::vector<real_type<T>>& d,
           std::vector<real_type<T>>& e, Reflectors<T>& QU, Reflectors<T>& QV, std::vector<T>& pu,
           std::vector<T>& pv);

/// Symmetric tridiagonal eigenproblem (d diagonal, e subdiagonal, n-1).
/// Eigenvalues ascending in d; when Z != nullptr its columns (zrows rows) are
/// multiplied by the eigenvector matrix (Z := Z * V).  Returns 0 or the
/// number of unconverged eigenvalues.
template <typename R, typename T>
int64_t steqr(int64_t n, R* d, R* e, T* Z, int64_t ldz, int64_t zrows);

template <typename R>
int64_t sterf(int64_t n, R* d, R* e);

/// Divide and conquer: eigenvalues ascending in d, eigenvectors in Q (n x n).
template <typename R>
int64_t stedc(int64_t n, R* d, R* e, R* Q, int64_t ldq);

// ---- the stages of stedc (reference stedc_solve.cc, stedc_z_vector.cc,
// stedc_sort.cc, stedc_deflate.cc, stedc_secular.cc, stedc_merge.cc)

/// Recursive D&C on the n x n tridiagonal (d, e[0:n-1]); Q gets its eigenvectors.
template <typename R>
void stedc_solve(int64_t n, R* d, R* e, R* Q, int64_t ldq);
/// Rank-one coupling vector z = [last row of Q1, sgn * first row of Q2] / sqrt(2)
/// of Q = diag(Q1 (n1 x n1), Q2).
template <typename R>
void stedc_z_vector(int64_t n1, int64_t n, R const* Q, int64_t ldq, R sgn, R* z);
/// Sort D ascending, permuting z and the columns of Q into Qp; perm[j] = source column.
template <typename R>
void stedc_sort(int64_t n, R* D, R* z, R const* Q, int64_t ldq, R* Qp, int64_t ldqp, int64_t* perm);
/// Deflation of D + rho z z^T: tiny z components and close D pairs (Givens on
/// Qp's columns).  deflated[j] = 1 marks deflated columns; returns the rest.
template <typename R>
int64_t stedc_deflate(int64_t n, R rho, R* D, R* z, R* Qp, int64_t ldqp, char* deflated);
/// Secular equation of D + rho z z^T (k x k, D ascending): eigenvalues lam
/// and orthonormal eigenvectors U (Gu-Eisenstat).
template <typename R>
void stedc_secular(int64_t k, R rho, R const* D, R const* z, R* lam, R* U, int64_t ldu);

/// Merge-product offload: C (m x n) = A (m x k) * B (k x n), element size
/// esize (4 or 8); installed by the device layer when a GPU is attached.
using StedcGemm = void (*)(size_t esize, int64_t m, int64_t n, int64_t k, const void* A, int64_t lda,
                           const void* B, int64_t ldb, void* C, int64_t ldc);
void set_stedc_gemm(StedcGemm f);

/// Bidiagonal SVD: B = diag(d) + superdiag(e) (n x n, upper).  Singular
/// values descending in d; U (urows x n) := U * Ub, VT (n x vcols) := Vb^T VT.
template <typename R, typename T>
int64_t bdsqr(int64_t n, R* d, R* e, T* U, int64_t ldu, int64_t urows, T* VT, int64_t ldvt, int64_t vcols);

/// Plane rotation on columns (i, i+1): [x y] <- [c x - s y, s x + c y].
template <typename R>
struct PlaneRot { int64_t i; R c, s; };

/// Where bdsqr's transformations go: U (rows x n) and Vt = VT^T (rows x n)
/// are only ever changed through these calls, so a device backend can batch
/// the sweeps and apply them on the GPU while the host iterates on (d, e).
template <typename R>
struct RotSink {
    virtual ~RotSink() = default;
    /// one implicit-shift QR sweep: adjacent rotations, ascending, on U (ru)
    /// and Vt (rv).  The sink may take the vectors' contents (swap); the
    /// caller clears them before the next sweep.
    virtual void sweep(std::vector<PlaneRot<R>>& ru, std::vector<PlaneRot<R>>& rv) = 0;
    /// cancellation rotation on U columns (a, b): [x y] <- [x c + y s, y c - x s]
    virtual void rot_u(int64_t a, int64_t b, R c, R s) = 0;
    /// Vt column k *= -1
    virtual void negate_v(int64_t k) = 0;
    /// final ordering: new column i = old column perm[i] (U and Vt)
    virtual void permute(std::vector<int64_t> const& perm) = 0;
};

/// bdsqr on (d, e) with every transformation sent to `sink` (may be null:
/// values only).  Returns the number of unconverged values.
template <typename R>
int64_t bdsqr_core(int64_t n, R* d, R* e, RotSink<R>* sink);

/// Implicit QL on (d, e) with every rotation sent to `sink` (sweep: the
/// sweep's rotations in application order, i descending; permute: the final
/// ascending sort).  Returns the number of unconverged eigenvalues.
template <typename R>
int64_t steqr_core(int64_t n, R* d, R* e, RotSink<R>* sink);

}  // namespace host
}  // namespace slate
