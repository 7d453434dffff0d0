// Local (per-process) BLAS/LAPACK layer: one entry point per operation that
// dispatches to the host C++ kernels (Target::Host*) or to the gfx950 device
// kernels on a HIP stream (Target::Devices).
//
// This is the counterpart of the reference's L3/L4 boundary: internal::X
// <Target> functions calling blas::batch::X / lapack::X per tile group
// (internal_gemm.cc:355-512, internal_herk.cc:351-530, internal_trsm.cc:132-255,
// internal_potrf.cc:56-80, internal_getrf_tntpiv.cc:325, internal_geqrf.cc:163-335).
// Because local storage is one strided array, each call here is ONE operation
// on the whole local block instead of a batch of tile operations.
#pragma once

#include "types.hh"
#include "comm.hh"
#include "device.hh"

namespace slate {
namespace lb {

/// Execution context: where to compute and, on the device, on which stream.
struct Ctx {
    Target target = Target::HostTask;
    hipStream_t stream = nullptr;
    bool dev() const { return target == Target::Devices; }
    Loc loc() const { return dev() ? Loc::Device : Loc::Host; }
    static Ctx host() { return Ctx{Target::HostTask, nullptr}; }
    static Ctx device(int queue) { return Ctx{Target::Devices, device::queue(queue)}; }
    Ctx on(int queue) const { return dev() ? device(queue) : *this; }
};

/// Per-stream scratch arena (stack discipline).  Memory released back to the
/// arena may be reused by later work on the SAME stream only, which stream
/// ordering makes safe; each stream has its own arena.
class Scratch {
public:
    explicit Scratch(Ctx const& ctx);
    ~Scratch();
    Scratch(Scratch const&) = delete;
    Scratch& operator=(Scratch const&) = delete;
    template <typename T> T* alloc(size_t n) { return static_cast<T*>(alloc_bytes(n * sizeof(T))); }
private:
    void* alloc_bytes(size_t bytes);
    Ctx ctx_;
    void* arena_;
    size_t mark_;
    std::vector<void*> host_;
};

// ---------------- BLAS-3
/// While alive on this thread, device NN gemms with K in (1000, 2048] and
/// m, n >= 8192 run as TN on a packed copy of A (SUMMA steps: the copy is
/// amortized over a large output; profiles/r6_gemm_pack_a_k.txt).
struct PackAHint {
    PackAHint();
    ~PackAHint();
    PackAHint(PackAHint const&) = delete;
    PackAHint& operator=(PackAHint const&) = delete;
};

template <typename T>
void gemm(Ctx const& c, Op opA, Op opB, int64_t m, int64_t n, int64_t k, T alpha,
          T const* A, int64_t lda, T const* B, int64_t ldb, T beta, T* C, int64_t ldc);

/// gemm as `splits` K-slices in one batched launch + in-order reduction of the
/// partials (real device types; otherwise plain gemm).  For short-wide
/// outputs with a long K (QR's W = V^H C): every workgroup stays short and the
/// slices fill the waves a handful of output tiles would leave idle.
template <typename T>
void gemm_splitk(Ctx const& c, Op opA, Op opB, int64_t m, int64_t n, int64_t k, int64_t splits, T alpha,
                 T const* A, int64_t lda, T const* B, int64_t ldb, T beta, T* C, int64_t ldc);

/// Right-hand-side counts up to which gemm (n columns, op(B) = B) and Left
/// trsm take the memory-bound gemv path on the device.
constexpr int64_t kSkinnyRhs = 16;

/// Y(m x nr) = alpha op(A) X + beta Y, op(A) m x k, X k x nr (device: gemv
/// kernels, K-chunked with an in-order partial reduction).
template <typename T>
void gemv(Ctx const& c, Op opA, int64_t m, int64_t k, int64_t nr, T alpha, T const* A, int64_t lda, T const* X,
          int64_t ldx, T beta, T* Y, int64_t ldy);

/// Triangle-only gemm: C(uplo) = alpha op(A) op(B) + beta C(uplo), C n x n.
template <typename T>
void gemm_tri(Ctx const& c, Uplo uplo, Op opA, Op opB, int64_t n, int64_t k, T alpha,
              T const* A, int64_t lda, T const* B, int64_t ldb, T beta, T* C, int64_t ldc);

/// C = alpha op(A) op(A)^H + beta C (herk) or ^T (syrk), uplo triangle.
template <typename T>
void herk(Ctx const& c, Uplo uplo, Op op, int64_t n, int64_t k, real_type<T> alpha,
          T const* A, int64_t lda, real_type<T> beta, T* C, int64_t ldc);
template <typename T>
void syrk(Ctx const& c, Uplo uplo, Op op, int64_t n, int64_t k, T alpha,
          T const* A, int64_t lda, T beta, T* C, int64_t ldc);
template <typename T>
void her2k(Ctx const& c, Uplo uplo, Op op, int64_t n, int64_t k, T alpha, T const* A, int64_t lda,
           T const* B, int64_t ldb, real_type<T> beta, T* C, int64_t ldc);
template <typename T>
void syr2k(Ctx const& c, Uplo uplo, Op op, int64_t n, int64_t k, T alpha, T const* A, int64_t lda,
           T const* B, int64_t ldb, T beta, T* C, int64_t ldc);
template <typename T>
void hemm(Ctx const& c, Side side, Uplo uplo, int64_t m, int64_t n, T alpha, T const* A, int64_t lda,
          T const* B, int64_t ldb, T beta, T* C, int64_t ldc, bool hermitian = true);
template <typename T>
void trsm(Ctx const& c, Side side, Uplo uplo, Op op, Diag diag, int64_t m, int64_t n, T alpha,
          T const* A, int64_t lda, T* B, int64_t ldb);
template <typename T>
void trmm(Ctx const& c, Side side, Uplo uplo, Op op, Diag diag, int64_t m, int64_t n, T alpha,
          T const* A, int64_t lda, T* B, int64_t ldb);

// ---------------- LAPACK-style
/// Cholesky of an n x n block; info (device int on Devices, host int on Host)
/// receives info_offset + failing column if not already set.
template <typename T>
void potrf(Ctx const& c, Uplo uplo, int64_t n, T* A, int64_t lda, int* info, int64_t info_offset);
/// Triangular inverse in place (uses a scratch copy on the device).
template <typename T>
void trtri(Ctx const& c, Uplo uplo, Diag diag, int64_t n, T* A, int64_t lda);
/// Inverse of triangular A into dense W (n x n, zeros outside the triangle).
template <typename T>
void trtri_to(Ctx const& c, Uplo uplo, Diag diag, int64_t n, T const* A, int64_t lda, T* W, int64_t ldw);
/// L^H L or U U^H in place.
template <typename T>
void lauum(Ctx const& c, Uplo uplo, int64_t n, T* A, int64_t lda);

/// LU with partial pivoting of an m x n panel (m >= n typical).  ipiv[j]
/// (device or host int64 array, length min(m,n)) receives the panel-relative
/// pivot row.  perm (length m) receives the resulting row permutation
/// (row t of the result is row perm[t] of the input) when non-null.
/// pivot=false gives LU without pivoting; tournament=true selects the pivots
/// of every 32-column narrow block by tournament (CALU) instead of per column.
/// pivot_threshold in (0, 1] (Option::PivotThreshold) keeps the diagonal entry
/// as pivot when |a_jj| >= threshold * max_i |a_ij| (1 = partial pivoting).
template <typename T>
void getrf_panel(Ctx const& c, int64_t m, int64_t n, T* A, int64_t lda, int64_t* ipiv, int64_t* perm,
                 int* info, int64_t info_offset, bool pivot = true, bool tournament = false,
                 double pivot_threshold = 1.0);

/// Apply a row permutation produced by getrf_panel (perm over the first m
/// rows, pivots ipiv[0..k)) to n columns of B.
template <typename T>
void apply_perm(Ctx const& c, int64_t k, int64_t const* perm, int64_t const* ipiv, int64_t n, T* B, int64_t ldb);

/// Householder QR of an m x n panel: V below the diagonal, R on/above, tau[n],
/// and the n x n upper-triangular block-reflector factor Tm (H = I - V T V^H).
template <typename T>
void geqrf_panel(Ctx const& c, int64_t m, int64_t n, T* A, int64_t lda, T* tau, T* Tm, int64_t ldt);

/// Apply H = I - V T V^H (op = ConjTrans applies H^H) from the left/right to
/// C (m x n); V given explicitly by `Vx` when non-null (unit diag, zeros above)
/// or taken from the lower trapezoid of V (diag implied 1).
template <typename T>
void larfb(Ctx const& c, Side side, Op op, int64_t m, int64_t n, int64_t k, T const* V, int64_t ldv,
           T const* Tm, int64_t ldt, T* C, int64_t ldc);

/// Explicit V (unit lower trapezoid) of an m x k factored panel into W (ld m).
template <typename T>
void form_v(Ctx const& c, int64_t m, int64_t k, T const* A, int64_t lda, T* W, int64_t ldw);

// ---------------- aux
template <typename T>
void set(Ctx const& c, Uplo uplo, int64_t m, int64_t n, T offdiag, T diag, T* A, int64_t lda);
template <typename Ts, typename Td>
void copy(Ctx const& c, Uplo uplo, Op op, int64_t m, int64_t n, Ts const* A, int64_t lda, Td* B, int64_t ldb);
template <typename T>
void add(Ctx const& c, Uplo uplo, int64_t m, int64_t n, T alpha, T const* A, int64_t lda, T beta, T* B, int64_t ldb);
template <typename T>
void scale(Ctx const& c, Uplo uplo, int64_t m, int64_t n, real_type<T> numer, real_type<T> denom, T* A, int64_t lda);
template <typename T>
void scale_row_col(Ctx const& c, int64_t m, int64_t n, real_type<T> const* R, real_type<T> const* Cs, T* A, int64_t lda);

/// Partial norms of a local block with global offsets (for trapezoid masks):
/// kind 'M' -> out[j] column max, '1' -> out[j] column abs sums,
/// 'I' -> out[i] row abs sums, 'F' -> out[2j..2j+1] (scale, sumsq).
/// `out` is a HOST array; device results are copied back (synchronizes).
template <typename T>
void norm_partial(Ctx const& c, char kind, Uplo uplo, Diag diag, int64_t m, int64_t n, T const* A, int64_t lda,
                  int64_t goff_row, int64_t goff_col, real_type<T>* out);

/// Copy between host and device or within a location (2-D strided).
template <typename T>
void copy2d(Ctx const& c, int64_t m, int64_t n, T const* src, int64_t lds, T* dst, int64_t ldd);

/// Throw if a persistent panel kernel reported a grid hand-off timeout since
/// the last check (synchronizes with the device).
void check_panel_errors();

}  // namespace lb
}  // namespace slate
