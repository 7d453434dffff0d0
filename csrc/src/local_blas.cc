// Local BLAS/LAPACK dispatch: host C++ kernels or gfx950 device kernels.
#include "slate_amd/local_blas.hh"
#include "slate_amd/host_blas.hh"
#include "../kernels/kernels.hh"
#include "slate_amd/eig_host.hh"

#include <map>
#include <mutex>
#include <cstring>
#include <cstdlib>

namespace slate {
namespace lb {

using slate_amd::dev::dptr;
using slate_amd::dev::dval;
namespace kd = slate_amd::dev;

//==============================================================================
// Scratch arenas
namespace {

struct Arena {
    struct Chunk { char* p; size_t size; };
    std::vector<Chunk> chunks;
    size_t cur = 0;      // current chunk index
    size_t off = 0;      // offset in current chunk
};

std::mutex g_arena_mtx;
std::map<hipStream_t, Arena>& arenas() {
    static auto* m = new std::map<hipStream_t, Arena>();
    return *m;
}

inline size_t align256(size_t b) { return (b + 255) / 256 * 256; }

}  // namespace

Scratch::Scratch(Ctx const& ctx) : ctx_(ctx), arena_(nullptr), mark_(0) {
    if (ctx_.dev()) {
        std::lock_guard<std::mutex> g(g_arena_mtx);
        Arena& a = arenas()[ctx_.stream];
        arena_ = &a;
        mark_ = (a.cur << 40) | a.off;
    }
}

Scratch::~Scratch() {
    if (ctx_.dev()) {
        std::lock_guard<std::mutex> g(g_arena_mtx);
        Arena& a = *static_cast<Arena*>(arena_);
        a.cur = mark_ >> 40;
        a.off = mark_ & ((size_t(1) << 40) - 1);
    }
    for (void* p : host_) std::free(p);
}

void* Scratch::alloc_bytes(size_t bytes) {
    bytes = align256(std::max<size_t>(bytes, 1));
    if (!ctx_.dev()) {
        void* p = nullptr;
        if (posix_memalign(&p, 256, bytes) != 0) throw std::bad_alloc();
        std::memset(p, 0, bytes);
        host_.push_back(p);
        return p;
    }
    std::lock_guard<std::mutex> g(g_arena_mtx);
    Arena& a = *static_cast<Arena*>(arena_);
    while (true) {
        if (a.cur < a.chunks.size()) {
            auto& c = a.chunks[a.cur];
            if (a.off + bytes <= c.size) {
                void* p = c.p + a.off;
                a.off += bytes;
                return p;
            }
            // try next chunk
            if (a.cur + 1 < a.chunks.size()) { a.cur++; a.off = 0; continue; }
        }
        // allocate a new chunk (at least 64 MiB, or twice the request)
        size_t sz = std::max<size_t>(size_t(64) << 20, 2 * bytes);
        char* p = static_cast<char*>(device::malloc(sz));
        a.chunks.push_back({p, sz});
        a.cur = a.chunks.size() - 1;
        a.off = 0;
    }
}

//==============================================================================
namespace {

inline char opc(Op op) { return char(op); }
inline char upc(Uplo u) { return char(u); }

template <typename T> constexpr bool is_real_v = !is_complex_v<T>;

// C = alpha op(A) op(B) + beta C as `splits` K-slices of one batched MFMA
// launch into partials P, then one in-order reduction (deterministic)
template <typename T>
void dgemm_splitk(hipStream_t s, char ta, char tb, int64_t m, int64_t n, int64_t k, int64_t splits, T alpha,
                  T const* A, int64_t lda, T const* B, int64_t ldb, T beta, T* C, int64_t ldc) {
    int64_t kc = roundup(ceildiv(k, splits), 16);
    splits = ceildiv(k, kc);
    int64_t full = k / kc;                 // chunks of exactly kc
    Scratch sc(Ctx{Target::Devices, s});
    T* P = sc.alloc<T>(size_t(splits) * m * n);
    int64_t sA = (ta == 'N') ? kc * lda : kc;
    int64_t sB = (tb == 'N') ? kc : kc * ldb;
    if (full > 0)
        kd::gemm_real<T>(ta, tb, m, n, kc, T(1), A, lda, sA, B, ldb, sB, T(0), P, m, m * n, full, s);
    if (full < splits) {
        int64_t krem = k - full * kc;
        kd::gemm_real<T>(ta, tb, m, n, krem, T(1), A + full * sA, lda, 0, B + full * sB, ldb, 0,
                         T(0), P + full * m * n, m, 0, 1, s);
    }
    kd::splitk_reduce<T>(m, n, int(splits), P, alpha, beta, C, ldc, s);
}

/// Does an NN product run as TN on a packed copy of A?  Always above K =
/// 2048; under a PackAHint (gemmC's SUMMA steps) also for K in
/// (SLATE_GEMM_PACK_A_MINK = 1000, 2048] when m, n >= 8192: the step GEMM
/// 32768 x 16384 x 2048 68.2 -> 69.2-69.7 TFLOP/s, 65536^2 x 1024 66.6 ->
/// 68.6, copies included; not for the factorizations' chunked updates
/// (dgeqrf 60.1 -> 59.8) (profiles/r6_gemm_pack_a_k.txt).  Otherwise NT on a
/// copy of B.
thread_local int t_pack_a_hint = 0;
inline int64_t pack_a_mink() {
    static const int64_t v = [] {
        const char* e = std::getenv("SLATE_GEMM_PACK_A_MINK");
        return e ? std::atoll(e) : int64_t(1000);
    }();
    return v;
}
inline bool pack_a_on() {
    static const bool v = [] {
        const char* e = std::getenv("SLATE_GEMM_PACK_A");
        return e ? std::atoi(e) != 0 : true;
    }();
    return v;
}
inline bool pack_a_form(int64_t m, int64_t n, int64_t k) {
    if (k > 2048) return m >= 4096 && n >= 4096;
    return t_pack_a_hint > 0 && k > pack_a_mink() && m >= 8192 && n >= 8192;
}
}  // namespace
slate::lb::PackAHint::PackAHint() { ++t_pack_a_hint; }
slate::lb::PackAHint::~PackAHint() { --t_pack_a_hint; }
namespace {
// SLATE_UPDATE_NT=0 keeps NN products in NN form (as internal::update_nt)
inline bool nt_pack() {
    static const bool v = [] {
        const char* e = std::getenv("SLATE_UPDATE_NT");
        return e ? std::atoi(e) != 0 : true;
    }();
    return v;
}

// device gemm dispatch (real -> MFMA, complex -> complex kernel)
template <typename T>
void dgemm(hipStream_t s, char uplo, Op opA, Op opB, int64_t m, int64_t n, int64_t k, T alpha,
           T const* A, int64_t lda, T const* B, int64_t ldb, T beta, T* C, int64_t ldc) {
    if (m <= 0 || n <= 0) return;
    if constexpr (is_real_v<T>) {
        char ta = opA == Op::NoTrans ? 'N' : 'T', tb = opB == Op::NoTrans ? 'N' : 'T';
        // split-K for small outputs with a long K (e.g. V^H C in QR panels):
        // otherwise only a handful of 128x128 tiles would carry all the work
        const int64_t tiles = ceildiv(m, 128) * ceildiv(n, 128);
        // (a handful of tiles with K >= 1024: the QR panel's V^H V and
        // V^H A products at the tail, where one workgroup would otherwise walk
        // all of K alone)
        if (tiles < 128 && k >= 1024) {
            // about 2 workgroups per CU in total and at most 64 partial
            // products, so the reduction stays a short streaming pass
            int64_t splits = std::min<int64_t>({ceildiv(k, 256), std::max<int64_t>(2, 512 / tiles), int64_t(64)});
            if (uplo == 'G') {
                dgemm_splitk(s, ta, tb, m, n, k, splits, alpha, A, lda, B, ldb, beta, C, ldc);
                return;
            }
            // triangular store (herk / syrk of a tall panel, e.g. the Gram
            // matrix of a CholeskyQR pass, K = 32768 x 512: 4.5 ms on 16
            // workgroups): the full product split over K into scratch, then
            // only the triangle merged into C
            Scratch sc(Ctx{Target::Devices, s});
            T* W = sc.alloc<T>(size_t(m) * n);
            dgemm_splitk(s, ta, tb, m, n, k, splits, T(1), A, lda, B, ldb, T(0), W, m);
            kd::geadd(uplo, m, n, dval(alpha), dptr(W), m, dval(beta), dptr(C), ldc, s);
            return;
        }
        // Rank-nb NN updates (SUMMA steps, K <= 2048): one transposed copy of
        // B (k x n -> n x k, a streaming pass of ~1/m of the product) turns
        // them into NT products on the 4-wave rotated tile, as the getrf /
        // geqrf trailing updates (same-box A/B, K = 512-1024: -1.7% time).
        // Not for long K: n = k = 65536 measured 68.7 (NN) -> 66.5 (NT)
        // TFLOP/s (profiles/r2_ab_prio_gemm_nt.txt).
        // (the copy is n x k <= n x 2048: bounded scratch, stream-ordered
        // reuse, so steady-state calls never reach hipMalloc)
        if (uplo == 'G' && ta == 'N' && tb == 'N' && sizeof(T) == 8 && nt_pack() && m >= 4096 &&
            n >= 1024 && k >= 256 && k <= 2048 && !(pack_a_on() && pack_a_form(m, n, k))) {
            const size_t bytes = size_t(n) * size_t(k) * sizeof(T);
            T* Bt = static_cast<T*>(device::malloc_async(bytes, s));
            kd::gecopy<T, T>('G', 'T', n, k, B, ldb, Bt, n, s);
            kd::gemm_real<T>('N', 'T', m, n, k, alpha, A, lda, 0, Bt, n, 0, beta, C, ldc, 0, 1, s);
            device::free_async(Bt, s);
            return;
        }
        // Long-K NN products as TN on a transposed copy of A (one streaming
        // pass): both operands K-contiguous, on the rotated 8-wave tile.
        // Same-box A/B at n = m = k = 65536 including the copy: 8172 -> 7900
        // ms, 68.9 -> 71.3 TFLOP/s (profiles/r2_ab_gemm_pack_a.txt); the NT
        // form (copy of B) measured slower there.  SLATE_GEMM_PACK_A=0: NN.
        // The copy is made in K slices of at most pack_bytes() (default
        // 8 GiB; later slices accumulate with beta = 1), so the scratch is
        // bounded independently of k and of the free HBM.
        if (pack_a_on() && uplo == 'G' && ta == 'N' && tb == 'N' && sizeof(T) == 8 && pack_a_form(m, n, k)) {
            const char* be = std::getenv("SLATE_GEMM_PACK_BYTES");
            const size_t budget = be ? size_t(std::atoll(be)) : (size_t(8) << 30);
            const int64_t kc = std::min<int64_t>(k, std::max<int64_t>(2048, int64_t(budget / (size_t(m) * sizeof(T))) / 256 * 256));
            T* At = static_cast<T*>(device::malloc_async(size_t(m) * size_t(kc) * sizeof(T), s));
            for (int64_t k0 = 0; k0 < k; k0 += kc) {
                const int64_t kk = std::min(kc, k - k0);
                kd::gecopy<T, T>('G', 'T', kk, m, A + k0 * lda, lda, At, kk, s);
                kd::gemm_real<T>('T', 'N', m, n, kk, alpha, At, kk, 0, B + k0, ldb, 0, k0 == 0 ? beta : T(1), C, ldc, 0,
                                 1, s);
            }
            device::free_async(At, s);
            return;
        }
        // K-chunked launches for large updates (SLATE_GEMM_KCHUNK): shorter
        // workgroups free CU slots for the high-priority panel queue sooner
        static const int64_t kchunk = [] {
            const char* e = std::getenv("SLATE_GEMM_KCHUNK");
            return e ? std::max<int64_t>(0, std::atoll(e)) : int64_t(0);
        }();
        const bool chunk = kchunk > 0 && k > kchunk && m * n >= int64_t(4096) * 4096;
        // k == 0 still runs once: C = beta C (BLAS semantics)
        for (int64_t k0 = 0; k0 < std::max<int64_t>(k, 1); k0 += chunk ? kchunk : std::max<int64_t>(k, 1)) {
            const int64_t kk = chunk ? std::min(kchunk, k - k0) : k;
            T const* Ak = A + (ta == 'N' ? k0 * lda : k0);
            T const* Bk = B + (tb == 'N' ? k0 : k0 * ldb);
            const T bk = k0 == 0 ? beta : T(1);
            if (uplo == 'G') kd::gemm_real<T>(ta, tb, m, n, kk, alpha, Ak, lda, 0, Bk, ldb, 0, bk, C, ldc, 0, 1, s);
            else {
                slate_assert(m == n);
                kd::gemm_tri_real<T>(uplo, ta, tb, n, kk, alpha, Ak, lda, Bk, ldb, bk, C, ldc, s);
            }
        }
    } else {
        kd::gemm_cplx(uplo, opc(opA), opc(opB), m, n, k, dval(alpha), dptr(A), lda, dptr(B), ldb,
                      dval(beta), dptr(C), ldc, s);
    }
}

template <typename T>
void dset(hipStream_t s, char uplo, int64_t m, int64_t n, T off, T diag, T* A, int64_t lda) {
    kd::geset(uplo, m, n, dval(off), dval(diag), dptr(A), lda, s);
}

template <typename T>
void dcopy(hipStream_t s, int64_t m, int64_t n, T const* A, int64_t lda, T* B, int64_t ldb) {
    if (m <= 0 || n <= 0) return;
    device::memcpy2d_async(B, ldb * sizeof(T), A, lda * sizeof(T), m * sizeof(T), n, s);
}

}  // namespace

//==============================================================================
// BLAS-3

template <typename T>
void gemm(Ctx const& c, Op opA, Op opB, int64_t m, int64_t n, int64_t k, T alpha,
          T const* A, int64_t lda, T const* B, int64_t ldb, T beta, T* C, int64_t ldc) {
    if (m <= 0 || n <= 0) return;
    if (!c.dev()) { host::gemm(opA, opB, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc); return; }
    if constexpr (is_real_v<T>) {
        // real: ConjTrans == Trans
        if (opA == Op::ConjTrans) opA = Op::Trans;
        if (opB == Op::ConjTrans) opB = Op::Trans;
    }
    if (n <= kSkinnyRhs && opB == Op::NoTrans) {
        // a few right-hand sides (residuals, refinement): memory-bound gemv
        // instead of 128-wide MFMA tiles with n live columns
        gemv(c, opA, m, k, n, alpha, A, lda, B, ldb, beta, C, ldc);
        return;
    }
    dgemm(c.stream, 'G', opA, opB, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc);
}

template <typename T>
void gemm_splitk(Ctx const& c, Op opA, Op opB, int64_t m, int64_t n, int64_t k, int64_t splits, T alpha,
                 T const* A, int64_t lda, T const* B, int64_t ldb, T beta, T* C, int64_t ldc) {
    if (m <= 0 || n <= 0) return;
    if constexpr (is_real_v<T>) {
        if (c.dev() && splits > 1 && k >= 2 * splits) {
            dgemm_splitk(c.stream, opA == Op::NoTrans ? 'N' : 'T', opB == Op::NoTrans ? 'N' : 'T', m, n, k, splits,
                         alpha, A, lda, B, ldb, beta, C, ldc);
            return;
        }
    }
    gemm(c, opA, opB, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc);
}

template <typename T>
void gemv(Ctx const& c, Op opA, int64_t m, int64_t k, int64_t nr, T alpha, T const* A, int64_t lda, T const* X,
          int64_t ldx, T beta, T* Y, int64_t ldy) {
    if (m <= 0 || nr <= 0) return;
    if (!c.dev()) { host::gemm(opA, Op::NoTrans, m, nr, k, alpha, A, lda, X, ldx, beta, Y, ldy); return; }
    const char tr = opA == Op::NoTrans ? 'N' : (opA == Op::Trans || is_real_v<T>) ? 'T' : 'C';
    const int chunks = kd::gemv_chunks(tr, m, k);
    Scratch sc(c);
    T* P = chunks > 1 ? sc.alloc<T>(size_t(chunks) * m * std::min<int64_t>(nr, kSkinnyRhs)) : nullptr;
    kd::gemv(tr, m, k, int(nr), dval(alpha), dptr(A), lda, dptr(X), ldx, dval(beta), dptr(Y), ldy, dptr(P), chunks,
             c.stream);
}

template <typename T>
void gemm_tri(Ctx const& c, Uplo uplo, Op opA, Op opB, int64_t n, int64_t k, T alpha,
              T const* A, int64_t lda, T const* B, int64_t ldb, T beta, T* C, int64_t ldc) {
    if (n <= 0) return;
    if (!c.dev()) {
        // compute full into temp and copy the triangle
        std::vector<T> W(size_t(n) * n);
        for (int64_t j = 0; j < n; ++j) for (int64_t i = 0; i < n; ++i) W[i + j * n] = C[i + j * ldc];
        host::gemm(opA, opB, n, n, k, alpha, A, lda, B, ldb, beta, W.data(), n);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < n; ++i)
                if (uplo == Uplo::Lower ? i >= j : i <= j) C[i + j * ldc] = W[i + j * n];
        return;
    }
    if constexpr (is_real_v<T>) {
        if (opA == Op::ConjTrans) opA = Op::Trans;
        if (opB == Op::ConjTrans) opB = Op::Trans;
    }
    dgemm(c.stream, upc(uplo), opA, opB, n, n, k, alpha, A, lda, B, ldb, beta, C, ldc);
}

template <typename T>
void herk(Ctx const& c, Uplo uplo, Op op, int64_t n, int64_t k, real_type<T> alpha,
          T const* A, int64_t lda, real_type<T> beta, T* C, int64_t ldc) {
    if (n <= 0) return;
    if (!c.dev()) { host::rankk(true, uplo, op, n, k, T(alpha), A, lda, T(beta), C, ldc); return; }
    // C = alpha op(A) op(A)^H: op = N -> A A^H ; op = C -> A^H A
    Op o1 = op == Op::NoTrans ? Op::NoTrans : Op::ConjTrans;
    Op o2 = op == Op::NoTrans ? Op::ConjTrans : Op::NoTrans;
    gemm_tri(c, uplo, o1, o2, n, k, T(alpha), A, lda, A, lda, T(beta), C, ldc);
}

template <typename T>
void syrk(Ctx const& c, Uplo uplo, Op op, int64_t n, int64_t k, T alpha,
          T const* A, int64_t lda, T beta, T* C, int64_t ldc) {
    if (n <= 0) return;
    if (!c.dev()) { host::rankk(false, uplo, op, n, k, alpha, A, lda, beta, C, ldc); return; }
    Op o1 = op == Op::NoTrans ? Op::NoTrans : Op::Trans;
    Op o2 = op == Op::NoTrans ? Op::Trans : Op::NoTrans;
    gemm_tri(c, uplo, o1, o2, n, k, alpha, A, lda, A, lda, beta, C, ldc);
}

template <typename T>
void her2k(Ctx const& c, Uplo uplo, Op op, int64_t n, int64_t k, T alpha, T const* A, int64_t lda,
           T const* B, int64_t ldb, real_type<T> beta, T* C, int64_t ldc) {
    if (n <= 0) return;
    if (!c.dev()) { host::rank2k(true, uplo, op, n, k, alpha, A, lda, B, ldb, T(beta), C, ldc); return; }
    Op o1 = op == Op::NoTrans ? Op::NoTrans : Op::ConjTrans;
    Op o2 = op == Op::NoTrans ? Op::ConjTrans : Op::NoTrans;
    gemm_tri(c, uplo, o1, o2, n, k, alpha, A, lda, B, ldb, T(beta), C, ldc);
    gemm_tri(c, uplo, o1, o2, n, k, slate::conj(alpha), B, ldb, A, lda, T(1), C, ldc);
}

template <typename T>
void syr2k(Ctx const& c, Uplo uplo, Op op, int64_t n, int64_t k, T alpha, T const* A, int64_t lda,
           T const* B, int64_t ldb, T beta, T* C, int64_t ldc) {
    if (n <= 0) return;
    if (!c.dev()) { host::rank2k(false, uplo, op, n, k, alpha, A, lda, B, ldb, beta, C, ldc); return; }
    Op o1 = op == Op::NoTrans ? Op::NoTrans : Op::Trans;
    Op o2 = op == Op::NoTrans ? Op::Trans : Op::NoTrans;
    gemm_tri(c, uplo, o1, o2, n, k, alpha, A, lda, B, ldb, beta, C, ldc);
    gemm_tri(c, uplo, o1, o2, n, k, alpha, B, ldb, A, lda, T(1), C, ldc);
}

template <typename T>
void hemm(Ctx const& c, Side side, Uplo uplo, int64_t m, int64_t n, T alpha, T const* A, int64_t lda,
          T const* B, int64_t ldb, T beta, T* C, int64_t ldc, bool hermitian) {
    if (m <= 0 || n <= 0) return;
    if (!c.dev()) { host::symm(hermitian, side, uplo, m, n, alpha, A, lda, B, ldb, beta, C, ldc); return; }
    // expand the symmetric/Hermitian block into a dense scratch copy, then gemm
    int64_t na = side == Side::Left ? m : n;
    Scratch sc(c);
    T* F = sc.alloc<T>(size_t(na) * na);
    dcopy(c.stream, na, na, A, lda, F, na);
    // G = full matrix: mirror (conj-)transpose of F, then the stored triangle
    T* G = sc.alloc<T>(size_t(na) * na);
    kd::gecopy('G', hermitian ? 'C' : 'T', na, na, dptr(F), na, dptr(G), na, c.stream);
    kd::gecopy(upc(uplo), 'N', na, na, dptr(F), na, dptr(G), na, c.stream);
    if (side == Side::Left) dgemm(c.stream, 'G', Op::NoTrans, Op::NoTrans, m, n, m, alpha, G, na, B, ldb, beta, C, ldc);
    else dgemm(c.stream, 'G', Op::NoTrans, Op::NoTrans, m, n, n, alpha, B, ldb, G, na, beta, C, ldc);
}

//------------------------------------------------------------------------------
template <typename T>
void trtri_to(Ctx const& c, Uplo uplo, Diag diag, int64_t n, T const* A, int64_t lda, T* W, int64_t ldw) {
    if (n <= 0) return;
    if (!c.dev()) {
        for (int64_t j = 0; j < n; ++j) for (int64_t i = 0; i < n; ++i) {
            bool in = uplo == Uplo::Lower ? i >= j : i <= j;
            W[i + j * ldw] = in ? A[i + j * lda] : T(0);
        }
        host::trtri(uplo, diag, n, W, ldw);
        return;
    }
    hipStream_t s = c.stream;
    constexpr int NBS = 64;
    dset(s, 'G', n, n, T(0), T(0), W, ldw);
    kd::trtri_diag(upc(uplo), char(diag), n, NBS, dptr(A), lda, dptr(W), ldw, s);
    Scratch sc(c);
    T* tmp = sc.alloc<T>(size_t(n) * n / 2 + NBS * NBS);
    for (int64_t sz = NBS; sz < n; sz *= 2) {
        int64_t p0 = 0;
        if constexpr (is_real_v<T>) {
            // the level's full-size pairs as two batched launches (they are
            // equally strided): fewer launches on the panel's critical path,
            // where each one waits for a CU slot behind the trailing GEMM
            static const bool batch = [] {
                const char* e = std::getenv("SLATE_TRTRI_BATCH");
                return e ? std::atoi(e) != 0 : true;
            }();
            const int64_t nfull = n / (2 * sz);
            if (batch && nfull >= 2) {
                const int64_t sa = 2 * sz * (1 + lda), sw = 2 * sz * (1 + ldw), st = sz * sz;
                if (uplo == Uplo::Lower) {
                    kd::gemm_real<T>('N', 'N', sz, sz, sz, T(1), A + sz, lda, sa, W, ldw, sw, T(0), tmp, sz, st,
                                     nfull, s);
                    kd::gemm_real<T>('N', 'N', sz, sz, sz, T(-1), W + sz + sz * ldw, ldw, sw, tmp, sz, st, T(0),
                                     W + sz, ldw, sw, nfull, s);
                } else {
                    kd::gemm_real<T>('N', 'N', sz, sz, sz, T(1), A + sz * lda, lda, sa, W + sz + sz * ldw, ldw, sw,
                                     T(0), tmp, sz, st, nfull, s);
                    kd::gemm_real<T>('N', 'N', sz, sz, sz, T(-1), W, ldw, sw, tmp, sz, st, T(0), W + sz * ldw, ldw,
                                     sw, nfull, s);
                }
                p0 = nfull * 2 * sz;
            }
        }
        for (int64_t p = p0; p + sz < n; p += 2 * sz) {
            int64_t s2 = std::min(sz, n - p - sz);
            if (uplo == Uplo::Lower) {
                // X21 = -X22 * A21 * X11 ; A21 = A[p+sz : +s2, p : +sz]
                dgemm(s, 'G', Op::NoTrans, Op::NoTrans, s2, sz, sz, T(1), A + (p + sz) + p * lda, lda,
                      W + p + p * ldw, ldw, T(0), tmp, s2);
                dgemm(s, 'G', Op::NoTrans, Op::NoTrans, s2, sz, s2, T(-1), W + (p + sz) + (p + sz) * ldw, ldw,
                      tmp, s2, T(0), W + (p + sz) + p * ldw, ldw);
            } else {
                // X12 = -X11 * A12 * X22 ; A12 = A[p : +sz, p+sz : +s2]
                dgemm(s, 'G', Op::NoTrans, Op::NoTrans, sz, s2, s2, T(1), A + p + (p + sz) * lda, lda,
                      W + (p + sz) + (p + sz) * ldw, ldw, T(0), tmp, sz);
                dgemm(s, 'G', Op::NoTrans, Op::NoTrans, sz, s2, sz, T(-1), W + p + p * ldw, ldw,
                      tmp, sz, T(0), W + p + (p + sz) * ldw, ldw);
            }
        }
    }
}

template <typename T>
void trtri(Ctx const& c, Uplo uplo, Diag diag, int64_t n, T* A, int64_t lda) {
    if (n <= 0) return;
    if (!c.dev()) { host::trtri(uplo, diag, n, A, lda); return; }
    Scratch sc(c);
    T* W = sc.alloc<T>(size_t(n) * n);
    trtri_to(c, uplo, diag, n, A, lda, W, n);
    // copy back the triangle (keep the other triangle of A untouched)
    kd::gecopy(upc(uplo), 'N', n, n, dptr(W), n, dptr(A), lda, c.stream);
}

/// small-triangle Left solves in one launch (SLATE_SMALL_TRSM=0: the
/// inverse + GEMM path)
inline bool small_trsm() {
    static const bool v = [] {
        const char* e = std::getenv("SLATE_SMALL_TRSM");
        return e ? std::atoi(e) != 0 : true;
    }();
    return v;
}

/// Left triangular solve with a few right-hand sides (n <= kSkinnyRhs):
/// every full BS x BS diagonal block inverted at once (batched doubling
/// GEMMs), then per block one gemv with the inverse and one gemv update of
/// the remaining rows -- about 5 launches per block instead of ~20 to
/// re-invert each block, and no 128-wide MFMA tiles carrying n live columns.
/// Returns false (caller falls back) for triangles shorter than two blocks.
template <typename T>
bool trsm_skinny(Ctx const& c, Uplo uplo, Op op, Diag diag, int64_t m, int64_t n, T const* A, int64_t lda, T* B,
                 int64_t ldb) {
    const int64_t BS = m >= 16384 ? 1024 : 512;
    const int64_t nfull = m / BS, rem = m - nfull * BS;
    if (nfull < 2) return false;
    hipStream_t s = c.stream;
    Scratch sc(c);
    T* Dinv = sc.alloc<T>(size_t(nfull) * BS * BS + size_t(rem) * rem);
    {
        Scratch sw(c);
        T* work = sw.alloc<T>(size_t(nfull) * BS * BS / 2);
        kd::trtri_blocks<T>(upc(uplo), char(diag), BS, nfull, A, lda, Dinv, work, s);
    }
    T* Drem = Dinv + size_t(nfull) * BS * BS;
    if (rem > 0) trtri_to(c, uplo, diag, rem, A + nfull * BS * (1 + lda), lda, Drem, rem);
    T* X = sc.alloc<T>(size_t(BS) * n);
    const bool lower_eff = (uplo == Uplo::Lower) == (op == Op::NoTrans);
    const int64_t nblk = nfull + (rem > 0);
    for (int64_t t = 0; t < nblk; ++t) {
        const int64_t bi = lower_eff ? t : nblk - 1 - t;
        const int64_t i0 = bi * BS, b = std::min(BS, m - i0);
        T const* D = bi < nfull ? Dinv + size_t(bi) * BS * BS : Drem;
        // x_t = op(A_tt)^{-1} b_t = op(A_tt^{-1}) b_t
        dcopy(s, b, n, B + i0, ldb, X, b);
        gemv(c, op, b, b, n, T(1), D, b, X, b, T(0), B + i0, ldb);
        // b_rest -= op(A)(rest, t) x_t
        const int64_t r0 = lower_eff ? i0 + b : 0, r1 = lower_eff ? m : i0;
        if (r1 > r0) {
            if (op == Op::NoTrans)
                gemv(c, op, r1 - r0, b, n, T(-1), A + r0 + i0 * lda, lda, B + i0, ldb, T(1), B + r0, ldb);
            else
                gemv(c, op, r1 - r0, b, n, T(-1), A + i0 + r0 * lda, lda, B + i0, ldb, T(1), B + r0, ldb);
        }
    }
    return true;
}

template <typename T>
void trsm(Ctx const& c, Side side, Uplo uplo, Op op, Diag diag, int64_t m, int64_t n, T alpha,
          T const* A, int64_t lda, T* B, int64_t ldb) {
    if (m <= 0 || n <= 0) return;
    if (!c.dev()) { host::trsm(side, uplo, op, diag, m, n, alpha, A, lda, B, ldb); return; }
    if constexpr (is_real_v<T>) { if (op == Op::ConjTrans) op = Op::Trans; }
    hipStream_t s = c.stream;
    if (alpha != T(1)) kd::geadd('G', m, n, dval(alpha), dptr(B), ldb, dval(T(0)), dptr(B), ldb, s);
    if (side == Side::Left && op == Op::NoTrans && m <= 64 && small_trsm()) {
        if (sizeof(T) == 4 && m > 32) {
            // fp32 64-row triangles as two 32-row solves and one GEMM: the
            // single 64-row fp32 launch measured ~2.5 ms per call beside the
            // fp32 trailing GEMM (profiles/r3_fp32_lu_trace.txt), the 32-row
            // one ~20 us
            const int64_t m1 = 32, m2 = m - 32;
            if (uplo == Uplo::Lower) {
                kd::trsm_small(upc(uplo), char(diag), int(m1), n, dptr(A), lda, dptr(B), ldb, s);
                dgemm(s, 'G', Op::NoTrans, Op::NoTrans, m2, n, m1, T(-1), A + m1, lda, B, ldb, T(1), B + m1, ldb);
                kd::trsm_small(upc(uplo), char(diag), int(m2), n, dptr(A + m1 + m1 * lda), lda, dptr(B + m1), ldb, s);
            } else {
                kd::trsm_small(upc(uplo), char(diag), int(m2), n, dptr(A + m1 + m1 * lda), lda, dptr(B + m1), ldb, s);
                dgemm(s, 'G', Op::NoTrans, Op::NoTrans, m1, n, m2, T(-1), A + m1 * lda, lda, B + m1, ldb, T(1), B, ldb);
                kd::trsm_small(upc(uplo), char(diag), int(m1), n, dptr(A), lda, dptr(B), ldb, s);
            }
            return;
        }
        kd::trsm_small(upc(uplo), char(diag), int(m), n, dptr(A), lda, dptr(B), ldb, s);
        return;
    }
    if constexpr (is_real_v<T>) {
        if (side == Side::Left && n <= kSkinnyRhs && trsm_skinny(c, uplo, op, diag, m, n, A, lda, B, ldb)) return;
    }
    const int64_t na = side == Side::Left ? m : n;
    const int64_t BS = 512;
    const bool lower_eff = (uplo == Uplo::Lower) == (op == Op::NoTrans);
    Scratch sc(c);
    const int64_t bs0 = std::min(BS, na);
    T* Ainv = sc.alloc<T>(size_t(bs0) * bs0);
    T* W = sc.alloc<T>(size_t(side == Side::Left ? bs0 * n : m * bs0));
    int64_t nblk = ceildiv(na, BS);
    for (int64_t t = 0; t < nblk; ++t) {
        // Left: forward if lower_eff; Right: forward if !lower_eff
        bool forward = (side == Side::Left) ? lower_eff : !lower_eff;
        int64_t bi = forward ? t : nblk - 1 - t;
        int64_t i0 = bi * BS, b = std::min(BS, na - i0);
        trtri_to(c, uplo, diag, b, A + i0 + i0 * lda, lda, Ainv, b);
        if (side == Side::Left) {
            dcopy(s, b, n, B + i0, ldb, W, b);
            dgemm(s, 'G', op, Op::NoTrans, b, n, b, T(1), Ainv, b, W, b, T(0), B + i0, ldb);
            // remaining rows
            int64_t r0 = forward ? i0 + b : 0, r1 = forward ? na : i0;
            if (r1 > r0) {
                if (op == Op::NoTrans)
                    dgemm(s, 'G', Op::NoTrans, Op::NoTrans, r1 - r0, n, b, T(-1), A + r0 + i0 * lda, lda,
                          B + i0, ldb, T(1), B + r0, ldb);
                else
                    dgemm(s, 'G', op, Op::NoTrans, r1 - r0, n, b, T(-1), A + i0 + r0 * lda, lda,
                          B + i0, ldb, T(1), B + r0, ldb);
            }
        } else {
            dcopy(s, m, b, B + i0 * ldb, ldb, W, m);
            dgemm(s, 'G', Op::NoTrans, op, m, b, b, T(1), W, m, Ainv, b, T(0), B + i0 * ldb, ldb);
            int64_t r0 = forward ? i0 + b : 0, r1 = forward ? na : i0;
            if (r1 > r0) {
                if (op == Op::NoTrans)
                    dgemm(s, 'G', Op::NoTrans, Op::NoTrans, m, r1 - r0, b, T(-1), B + i0 * ldb, ldb,
                          A + i0 + r0 * lda, lda, T(1), B + r0 * ldb, ldb);
                else
                    dgemm(s, 'G', Op::NoTrans, op, m, r1 - r0, b, T(-1), B + i0 * ldb, ldb,
                          A + r0 + i0 * lda, lda, T(1), B + r0 * ldb, ldb);
            }
        }
    }
}

template <typename T>
void trmm(Ctx const& c, Side side, Uplo uplo, Op op, Diag diag, int64_t m, int64_t n, T alpha,
          T const* A, int64_t lda, T* B, int64_t ldb) {
    if (m <= 0 || n <= 0) return;
    if (!c.dev()) { host::trmm(side, uplo, op, diag, m, n, alpha, A, lda, B, ldb); return; }
    if constexpr (is_real_v<T>) { if (op == Op::ConjTrans) op = Op::Trans; }
    hipStream_t s = c.stream;
    int64_t na = side == Side::Left ? m : n;
    Scratch sc(c);
    T* F = sc.alloc<T>(size_t(na) * na);
    T* W = sc.alloc<T>(size_t(m) * n);
    // dense triangle with explicit zeros; unit diagonal set by walking the
    // diagonal as a 1 x na view with ld = na + 1
    dset(s, 'G', na, na, T(0), T(0), F, na);
    kd::gecopy(upc(uplo), 'N', na, na, dptr(A), lda, dptr(F), na, s);
    if (diag == Diag::Unit) dset(s, 'G', 1, na, T(1), T(1), F, na + 1);
    dcopy(s, m, n, B, ldb, W, m);
    if (side == Side::Left) dgemm(s, 'G', op, Op::NoTrans, m, n, m, alpha, F, na, W, m, T(0), B, ldb);
    else dgemm(s, 'G', Op::NoTrans, op, m, n, n, alpha, W, m, F, na, T(0), B, ldb);
}

//------------------------------------------------------------------------------
template <typename T>
void potrf(Ctx const& c, Uplo uplo, int64_t n, T* A, int64_t lda, int* info, int64_t info_offset) {
    if (n <= 0) return;
    if (!c.dev()) {
        int64_t r = host::potrf(uplo, n, A, lda);
        if (r != 0 && info && *info == 0) *info = int(info_offset + r);
        return;
    }
    constexpr int64_t NB0 = 64;
    // Two launches per leaf (sizeof(T) <= 8: the leaf kernel's per-lane row
    // fits in 128 VGPRs): factor + A21 solve in one kernel, then the trailing
    // triangle.  SLATE_POTRF_LEAF=0 keeps the inverse-based leaf.
    static const bool leaf = [] {
        const char* e = std::getenv("SLATE_POTRF_LEAF");
        return e ? std::atoi(e) != 0 : true;
    }();
    const bool use_leaf = sizeof(T) <= 8 && leaf && uplo == Uplo::Lower;
    if (n <= NB0) {
        if (use_leaf)
            kd::potrf_leaf<kd::dev_t<T>>(int(n), 0, dptr(A), lda, info, int(info_offset), nullptr, nullptr, nullptr, 0,
                                     c.stream);
        else kd::potrf_small(upc(uplo), int(n), dptr(A), lda, info, int(info_offset), c.stream);
        return;
    }
    static const bool blocked = [] {
        const char* e = std::getenv("SLATE_POTRF_BLOCKED");
        return e ? std::atoi(e) != 0 : true;
    }();
    // Above rec_max columns the recursive split below runs first (its trsm /
    // herk at the top levels are large GEMMs), the blocked 64-column sweep
    // only on the blocks of at most rec_max: the 1x1 potrf's tail (8192
    // columns, potrf.cc) as one 128-leaf sweep ran its rank-64 updates at
    // ~9 TFLOP/s.  SLATE_POTRF_REC_MAX (0: always blocked, the default:
    // config 2 measured 48.9 TFLOP/s all-blocked against 48.1 / 48.6 at 1024 /
    // 2048 -- the recursion's own trsm / herk chain costs what the larger
    // GEMMs save; profiles/r4_lu_split_potrf_rec.txt).
    static const int64_t rec_max = [] {
        const char* e = std::getenv("SLATE_POTRF_REC_MAX");
        return e ? std::atoll(e) : int64_t(0);
    }();
    if (uplo == Uplo::Lower && blocked && (rec_max <= 0 || n <= rec_max)) {
        // Right-looking over 64-column leaves, four launches per leaf: the
        // leaf's factor and its inverse in one kernel, the rows below as one
        // GEMM with the inverse (into Y), the trailing triangle as one
        // triangular GEMM from Y, Y copied back.  The recursive form below
        // re-inverts every off-diagonal level's triangle (~50 launches for
        // n = 512 against ~29 here); on the factorization's critical path
        // each launch waits for a CU slot behind the trailing update.
        hipStream_t s = c.stream;
        if (use_leaf) {
            // L11 of leaf k is staged in Wk[k & 1] and copied into A by leaf k+1
            Scratch sc(c);
            T* Wk[2] = {sc.alloc<T>(size_t(NB0) * NB0), sc.alloc<T>(size_t(NB0) * NB0)};
            T* Aprev = nullptr;
            int bprev = 0;
            for (int64_t j0 = 0, k = 0; j0 < n; j0 += NB0, ++k) {
                const int64_t b = std::min(NB0, n - j0), r = n - j0 - b;
                T* Ajj = A + j0 + j0 * lda;
                kd::potrf_leaf<kd::dev_t<T>>(int(b), r, dptr(Ajj), lda, info, int(info_offset + j0), dptr(Wk[k & 1]),
                                         Aprev ? dptr(Wk[(k + 1) & 1]) : nullptr, dptr(Aprev), bprev, s);
                Aprev = Ajj;
                bprev = int(b);
                if (r == 0) break;
                T* Ab = Ajj + b;
                dgemm(s, 'L', Op::NoTrans, Op::ConjTrans, r, r, b, T(-1), Ab, lda, Ab, lda, T(1), Ab + b * lda, lda);
            }
            return;
        }
        Scratch sc(c);
        T* Winv = sc.alloc<T>(size_t(NB0) * NB0);
        T* Y = sc.alloc<T>(size_t(n) * NB0);
        for (int64_t j0 = 0; j0 < n; j0 += NB0) {
            const int64_t b = std::min(NB0, n - j0), r = n - j0 - b;
            T* Ajj = A + j0 + j0 * lda;
            kd::potrf_inv_small(int(b), dptr(Ajj), lda, dptr(Winv), NB0, info, int(info_offset + j0), s);
            if (r == 0) break;
            T* Ab = Ajj + b;
            dgemm(s, 'G', Op::NoTrans, Op::ConjTrans, r, b, b, T(1), Ab, lda, Winv, NB0, T(0), Y, r);
            dgemm(s, 'L', Op::NoTrans, Op::ConjTrans, r, r, b, T(-1), Y, r, Y, r, T(1), Ab + b * lda, lda);
            dcopy(s, r, b, Y, r, Ab, lda);
        }
        return;
    }
    int64_t n1 = roundup(ceildiv(n, 2), NB0), n2 = n - n1;
    potrf(c, uplo, n1, A, lda, info, info_offset);
    if (uplo == Uplo::Lower) {
        trsm(c, Side::Right, Uplo::Lower, Op::ConjTrans, Diag::NonUnit, n2, n1, T(1), A, lda, A + n1, lda);
        herk(c, Uplo::Lower, Op::NoTrans, n2, n1, real_type<T>(-1), A + n1, lda, real_type<T>(1), A + n1 + n1 * lda, lda);
    } else {
        trsm(c, Side::Left, Uplo::Upper, Op::ConjTrans, Diag::NonUnit, n1, n2, T(1), A, lda, A + n1 * lda, lda);
        herk(c, Uplo::Upper, Op::ConjTrans, n2, n1, real_type<T>(-1), A + n1 * lda, lda, real_type<T>(1), A + n1 + n1 * lda, lda);
    }
    potrf(c, uplo, n2, A + n1 + n1 * lda, lda, info, info_offset + n1);
}

template <typename T>
void lauum(Ctx const& c, Uplo uplo, int64_t n, T* A, int64_t lda) {
    if (n <= 0) return;
    if (!c.dev()) { host::lauum(uplo, n, A, lda); return; }
    Scratch sc(c);
    T* F = sc.alloc<T>(size_t(n) * n);
    dset(c.stream, 'G', n, n, T(0), T(0), F, n);
    kd::gecopy(upc(uplo), 'N', n, n, dptr(A), lda, dptr(F), n, c.stream);
    if (uplo == Uplo::Lower)
        gemm_tri(c, Uplo::Lower, Op::ConjTrans, Op::NoTrans, n, n, T(1), F, n, F, n, T(0), A, lda);
    else
        gemm_tri(c, Uplo::Upper, Op::NoTrans, Op::ConjTrans, n, n, T(1), F, n, F, n, T(0), A, lda);
}

//------------------------------------------------------------------------------
// LU panel
namespace {

template <typename T>
struct LuPanelDev {
    hipStream_t s;
    int64_t m, ncols;          // panel rows, panel width (swaps span all ncols)
    T* A0; int64_t lda;
    int64_t* ipiv; int64_t* perm;
    int* info; int64_t info_offset;
    real_type<T>* pval; int64_t* pidx;
    bool pivot, tournament;
    double thresh;
    int64_t* tws;
    Ctx ctx;

    void narrow(int64_t c0, int64_t nn) {
        using DT = kd::dev_t<T>;
        DT* A = dptr(A0);
        int64_t kmax = std::min(nn, m - c0);
        if (kmax <= 0) return;
        if (tournament && pivot && m - c0 >= 2 * nn) {
            kd::tslu_narrow<DT>(m, c0, int(kmax), A + c0 * lda, A, lda, ncols, ipiv, perm, info, info_offset, tws, s);
            return;
        }
        int nparts = int(ceildiv(m - c0, 256));
        if (pivot) kd::lu_colmax<DT>(m, c0, A, lda, c0, pval, pidx, nparts, s);
        for (int64_t j = 0; j < kmax; ++j) {
            int64_t col = c0 + j;
            kd::lu_pivot<DT>(pivot ? nparts : 0, pval, pidx, col, col, A, lda, ncols, ipiv, 0, perm, info,
                             info_offset, nullptr, s, thresh);
            // update columns (col, c0+nn); deferred scaling of column col-1
            kd::lu_update2d<DT>(m, col, col, c0 + nn, A, lda, pval, pidx, j > 0 ? 1 : 0, s);
            nparts = int(ceildiv(m - col, 256));
        }
        kd::lu_scale_col<DT>(m, c0 + kmax - 1, A, lda, s);
    }

    void rec(int64_t c0, int64_t nn) {
        constexpr int64_t W = 32;
        if (c0 >= m) return;
        if (nn <= W) { narrow(c0, nn); return; }
        int64_t n1 = roundup(ceildiv(nn, 2), W), n2 = nn - n1;
        rec(c0, n1);
        if (c0 + n1 > m) return;
        // U12 = L11^{-1} A12 ; A22 -= L21 U12
        trsm(ctx, Side::Left, Uplo::Lower, Op::NoTrans, Diag::Unit, n1, n2, T(1),
             A0 + c0 + c0 * lda, lda, A0 + c0 + (c0 + n1) * lda, lda);
        dgemm(s, 'G', Op::NoTrans, Op::NoTrans, m - c0 - n1, n2, n1, T(-1),
              A0 + (c0 + n1) + c0 * lda, lda, A0 + c0 + (c0 + n1) * lda, lda, T(1),
              A0 + (c0 + n1) + (c0 + n1) * lda, lda);
        rec(c0 + n1, n2);
    }
};

}  // namespace

template <typename T>
void getrf_panel(Ctx const& c, int64_t m, int64_t n, T* A, int64_t lda, int64_t* ipiv, int64_t* perm,
                 int* info, int64_t info_offset, bool pivot, bool tournament, double pivot_threshold) {
    if (m <= 0 || n <= 0) return;
    if (!c.dev()) {
        std::vector<int64_t> piv(std::min(m, n));
        int64_t r = host::getrf(m, n, A, lda, piv.data(), pivot, pivot_threshold);
        if (r != 0 && info && *info == 0) *info = int(info_offset + r);
        for (size_t j = 0; j < piv.size(); ++j) ipiv[j] = piv[j];
        if (perm) {
            for (int64_t i = 0; i < m; ++i) perm[i] = i;
            for (size_t j = 0; j < piv.size(); ++j) std::swap(perm[j], perm[piv[j]]);
        }
        return;
    }
    Scratch sc(c);
    LuPanelDev<T> P;
    P.s = c.stream; P.m = m; P.ncols = n; P.A0 = A; P.lda = lda; P.ipiv = ipiv; P.perm = perm;
    P.info = info; P.info_offset = info_offset; P.pivot = pivot; P.tournament = tournament; P.ctx = c;
    P.thresh = pivot_threshold;
    P.tws = tournament ? sc.alloc<int64_t>(size_t(kd::tslu_workspace(m))) : nullptr;
    if (P.tws) kd::tslu_init(P.tws, c.stream);
    int64_t np = ceildiv(m, 256) + 1;
    P.pval = sc.alloc<real_type<T>>(np);
    P.pidx = sc.alloc<int64_t>(np);
    if (perm) kd::iota(m, perm, c.stream);
    P.rec(0, std::min(m, n));
    // columns beyond min(m,n) (wide panel): U12 = L11^{-1} A12
    if (n > m)
        trsm(c, Side::Left, Uplo::Lower, Op::NoTrans, Diag::Unit, m, n - m, T(1), A, lda, A + m * lda, lda);
}

template <typename T>
void apply_perm(Ctx const& c, int64_t k, int64_t const* perm, int64_t const* ipiv, int64_t n, T* B, int64_t ldb) {
    if (k <= 0 || n <= 0) return;
    if (!c.dev()) {
        // rows [0, k) and pivot rows: new[t] = old[perm[t]]
        std::vector<int64_t> rows;
        for (int64_t t = 0; t < k; ++t) rows.push_back(t);
        for (int64_t t = 0; t < k; ++t) if (ipiv[t] >= k) rows.push_back(ipiv[t]);
        std::vector<T> tmp(rows.size());
        for (int64_t j = 0; j < n; ++j) {
            T* col = B + j * ldb;
            for (size_t r = 0; r < rows.size(); ++r) tmp[r] = col[perm[rows[r]]];
            for (size_t r = 0; r < rows.size(); ++r) col[rows[r]] = tmp[r];
        }
        return;
    }
    Scratch sc(c);
    int64_t* dst = sc.alloc<int64_t>(2 * k);
    int64_t* src = sc.alloc<int64_t>(2 * k);
    kd::perm_pairs(k, perm, ipiv, dst, src, c.stream);
    kd::permute_rows(n, dptr(B), ldb, dst, src, nullptr, int(2 * k), c.stream);
}

//------------------------------------------------------------------------------
// QR panel
template <typename T>
void form_v(Ctx const& c, int64_t m, int64_t k, T const* A, int64_t lda, T* W, int64_t ldw) {
    if (m <= 0 || k <= 0) return;
    if (!c.dev()) {
        for (int64_t j = 0; j < k; ++j)
            for (int64_t i = 0; i < m; ++i)
                W[i + j * ldw] = i < j ? T(0) : (i == j ? T(1) : A[i + j * lda]);
        return;
    }
    kd::form_v(m, k, int64_t(0), dptr(A), lda, dptr(W), ldw, c.stream);
}

template <typename T>
void larfb(Ctx const& c, Side side, Op op, int64_t m, int64_t n, int64_t k, T const* V, int64_t ldv,
           T const* Tm, int64_t ldt, T* C, int64_t ldc) {
    if (m <= 0 || n <= 0 || k <= 0) return;
    if (!c.dev()) { host::larfb(side, op, m, n, k, V, ldv, Tm, ldt, C, ldc); return; }
    hipStream_t s = c.stream;
    Scratch sc(c);
    int64_t mv = side == Side::Left ? m : n;
    T* Vx = sc.alloc<T>(size_t(mv) * k);
    form_v(c, mv, k, V, ldv, Vx, mv);
    Op tOp = op == Op::NoTrans ? Op::NoTrans : Op::ConjTrans;
    if constexpr (is_real_v<T>) { if (tOp == Op::ConjTrans) tOp = Op::Trans; }
    Op cT = is_complex_v<T> ? Op::ConjTrans : Op::Trans;
    if (side == Side::Left) {
        T* W = sc.alloc<T>(size_t(k) * n);
        T* W2 = sc.alloc<T>(size_t(k) * n);
        // W = V^H C (k x n, K = m): tall-skinny when n small
        if (n <= 32 && k <= 32) {   // tsip handles m, n <= 32
            T* work = sc.alloc<T>(size_t(1) << 20);
            kd::tsip(m, int(k), int(n), dval(T(1)), dptr(Vx), mv, dptr(C), ldc, dval(T(0)), dptr(W), k,
                     dptr(work), int64_t(1) << 20, s);
        } else {
            dgemm(s, 'G', cT, Op::NoTrans, k, n, m, T(1), Vx, mv, C, ldc, T(0), W, k);
        }
        dgemm(s, 'G', tOp, Op::NoTrans, k, n, k, T(1), Tm, ldt, W, k, T(0), W2, k);
        dgemm(s, 'G', Op::NoTrans, Op::NoTrans, m, n, k, T(-1), Vx, mv, W2, k, T(1), C, ldc);
    } else {
        T* W = sc.alloc<T>(size_t(m) * k);
        T* W2 = sc.alloc<T>(size_t(m) * k);
        dgemm(s, 'G', Op::NoTrans, Op::NoTrans, m, k, n, T(1), C, ldc, Vx, mv, T(0), W, m);
        dgemm(s, 'G', Op::NoTrans, tOp, m, k, k, T(1), W, m, Tm, ldt, T(0), W2, m);
        dgemm(s, 'G', Op::NoTrans, cT, m, n, k, T(-1), W2, m, Vx, mv, T(1), C, ldc);
    }
}

namespace {

/// Device word set by persistent panel kernels when a grid hand-off times out.
unsigned* panel_error_word() {
    static unsigned* w = [] {
        auto* p = static_cast<unsigned*>(device::malloc(256));
        slate_hip_call(hipMemset(p, 0, 256));
        return p;
    }();
    return w;
}

template <typename T>
struct QrPanelDev {
    hipStream_t s;
    int64_t m;
    T* A0; int64_t lda;
    T* tau;
    T* Tm; int64_t ldt;
    Ctx ctx;
    real_type<T>* psum; T* alpha; T* pdots; T* work; int64_t work_elems; T* scal;
    T* tsqr_work = nullptr;
    // explicit unit-lower V of the whole panel (ld m), filled once per narrow
    // block: the recursion's larfb / merge GEMMs read it directly instead of
    // forming V again (copy + triangle set) at every level
    T* Vp = nullptr; int64_t ldvp = 0;

    // (all m rows of the block's columns: the zeros above its diagonal are
    // read by the outer levels' products, whose V spans several blocks)
    void keep_v(int64_t c0, int64_t kmax) {
        kd::form_v(m, kmax, c0, dptr(A0 + c0 * lda), lda, dptr(Vp + c0 * ldvp), ldvp, s);
    }

    // narrow block [c0, c0+nn): Householder columns + T block (nn x nn at Tm[c0, c0])
    void narrow(int64_t c0, int64_t nn) {
        using DT = kd::dev_t<T>;
        DT* A = dptr(A0);
        int64_t kmax = std::min(nn, m - c0);
        if (kmax <= 0) return;
        if (use_tsqr(c0, nn)) {
            // on-chip TSQR tree + Householder reconstruction (tsqr.hip): about
            // 2 log8(rows/256) + 4 launches per narrow block instead of two per column
            kd::qr_tsqr_narrow<DT>(m - c0, int(nn), A + c0 + c0 * lda, lda, dptr(Tm + c0 + c0 * ldt), ldt,
                                   dptr(tau + c0), dptr(tsqr_work), s);
            keep_v(c0, kmax);
            return;
        }
        if (use_persistent(c0)) {
            // one launch for the whole block, LDS-resident (qr_persistent.hip)
            Scratch sc(ctx);
            int G = kd::qr_narrow_groups<DT>(m - c0);
            auto* part = sc.alloc<unsigned long long>(kd::qr_narrow_workspace_words(G));
            auto* cnt = sc.alloc<unsigned>(32);
            kd::qr_narrow<DT>(m, c0, int(nn), A, lda, dptr(tau), part, cnt, panel_error_word(), s);
        } else {
            columns(c0, nn, kmax);
        }
        t_block(c0, kmax);
    }

    // Opt-in (SLATE_QR_PANEL=persistent): measured 21.9 ms vs 18.2 ms for the
    // two-launch column path on a 65536 x 512 panel in isolation (one grid
    // hand-off per column is ~30 us: three round trips to the coherence
    // point), and slower still under a concurrent trailing GEMM, which delays
    // co-residency of the 128 workgroups.  Kept for panels that do fit one
    // XCD / for future fused variants.
    // SLATE_QR_PANEL=columns selects the column-at-a-time path (A/B runs)
    static bool tsqr_enabled() {
        static int on = [] { const char* e = std::getenv("SLATE_QR_PANEL"); return !(e && (std::string(e) == "columns" || std::string(e) == "persistent")); }();
        return on;
    }
    // (rows > nn: a square last block keeps the column path, whose last
    // reflector is the identity exactly as in LAPACK, so R's sign convention
    // matches the host path on every block)
    // (real types: the complex node kernel does not fit its block in VGPRs)
    bool use_tsqr(int64_t c0, int64_t nn) const {
        return is_real_v<T> && tsqr_enabled() && m - c0 > nn && nn <= 32;
    }
    static bool persistent_enabled() {
        static int on = [] { const char* e = std::getenv("SLATE_QR_PANEL"); return e && std::string(e) == "persistent"; }();
        return on;
    }
    // real types whose block fits the persistent kernel's grid (<= 160 resident workgroups)
    bool use_persistent(int64_t c0) const {
        if (!persistent_enabled() || is_complex_v<T>) return false;
        return kd::qr_narrow_groups<kd::dev_t<T>>(m - c0) <= 160;
    }

    // column-at-a-time path: two stream-ordered launches per column
    void columns(int64_t c0, int64_t nn, int64_t kmax) {
        using DT = kd::dev_t<T>;
        DT* A = dptr(A0);
        int nparts = int(std::max<int64_t>(1, ceildiv(m - c0 - 1, 256)));
        kd::qr_colnorm<DT>(m, c0, A, lda, c0, psum, dptr(alpha), nparts, s);
        for (int64_t j = 0; j < kmax; ++j) {
            int64_t col = c0 + j;
            int nblk = int(ceildiv(m - col, 256));
            kd::qr_dots2d<DT>(m, col, col, c0 + nn, A, lda, nparts, psum, dptr(alpha), dptr(tau), dptr(scal),
                              dptr(pdots), j > 0 ? 1 : 0, s);
            kd::qr_update2d<DT>(m, col, col, c0 + nn, A, lda, nblk, dptr(pdots), dptr(tau), dptr(scal), psum,
                                dptr(alpha), s);
            nparts = nblk;
        }
        kd::qr_scale_col<DT>(m, c0 + kmax - 1, A, lda, dptr(scal), s);
    }

    // T block of the narrow block: S = V^H V then the larft recurrence
    void t_block(int64_t c0, int64_t kmax) {
        int64_t mv = m - c0;
        keep_v(c0, kmax);
        T* Vx = Vp + c0 + c0 * ldvp;
        T* Tb = Tm + c0 + c0 * ldt;
        kd::tsip(mv, int(kmax), int(kmax), dval(T(1)), dptr(Vx), ldvp, dptr(Vx), ldvp, dval(T(0)), dptr(Tb), ldt,
                 dptr(work), work_elems, s);
        kd::larft_small(int(kmax), dptr(tau + c0), dptr(Tb), ldt, s);
    }

    // C -= V T^H V^H C for the panel's block [c0, c0 + k) applied to
    // columns [cc, cc + n) (V explicit in Vp)
    void apply_left(int64_t c0, int64_t k, int64_t cc, int64_t n) {
        const int64_t mv = m - c0;
        if (mv <= 0 || n <= 0 || k <= 0) return;
        Scratch sc(ctx);
        const Op cT = is_complex_v<T> ? Op::ConjTrans : Op::Trans;
        T const* V = Vp + c0 + c0 * ldvp;
        T* C = A0 + c0 + cc * lda;
        T* W = sc.alloc<T>(size_t(k) * n);
        T* W2 = sc.alloc<T>(size_t(k) * n);
        if (n <= 32 && k <= 32) {   // tsip handles m, n <= 32
            T* wk = sc.alloc<T>(size_t(1) << 20);
            kd::tsip(mv, int(k), int(n), dval(T(1)), dptr(V), ldvp, dptr(C), lda, dval(T(0)), dptr(W), k, dptr(wk),
                     int64_t(1) << 20, s);
        } else {
            dgemm(s, 'G', cT, Op::NoTrans, k, n, mv, T(1), V, ldvp, C, lda, T(0), W, k);
        }
        dgemm(s, 'G', cT, Op::NoTrans, k, n, k, T(1), Tm + c0 + c0 * ldt, ldt, W, k, T(0), W2, k);
        dgemm(s, 'G', Op::NoTrans, Op::NoTrans, mv, n, k, T(-1), V, ldvp, W2, k, T(1), C, lda);
    }

    void rec(int64_t c0, int64_t nn) {
        constexpr int64_t W = 32;
        if (c0 >= m) return;
        if (nn <= W) { narrow(c0, nn); return; }
        int64_t n1 = roundup(ceildiv(nn, 2), W), n2 = nn - n1;
        rec(c0, n1);
        // apply H1^H to the right columns
        apply_left(c0, std::min(n1, m - c0), c0 + n1, n2);
        rec(c0 + n1, n2);
        if (c0 + n1 >= m) return;
        // merge: T12 = -T11 (V1^H V2) T22, V1 rows from c0+n1, V2 rows from c0+n1
        int64_t k2 = std::min(n2, m - c0 - n1);
        Scratch sc(ctx);
        int64_t mv = m - c0 - n1;
        T const* V2 = Vp + (c0 + n1) + (c0 + n1) * ldvp;
        T* S = sc.alloc<T>(size_t(n1) * k2);
        Op cT = is_complex_v<T> ? Op::ConjTrans : Op::Trans;
        // V1 rows [c0+n1, m) are plain stored (below V1's diagonal block)
        dgemm(s, 'G', cT, Op::NoTrans, n1, k2, mv, T(1), A0 + (c0 + n1) + c0 * lda, lda, V2, ldvp, T(0), S, n1);
        T* S2 = sc.alloc<T>(size_t(n1) * k2);
        dgemm(s, 'G', Op::NoTrans, Op::NoTrans, n1, k2, k2, T(1), S, n1, Tm + (c0 + n1) + (c0 + n1) * ldt, ldt,
              T(0), S2, n1);
        // T11 is stored upper triangular with explicit zeros below (narrow
        // blocks and merges write it so, and T starts zeroed): the trmm is a
        // plain GEMM straight into T12
        dgemm(s, 'G', Op::NoTrans, Op::NoTrans, n1, k2, n1, T(-1), Tm + c0 + c0 * ldt, ldt, S2, n1, T(0),
              Tm + c0 + (c0 + n1) * ldt, ldt);
    }
};

}  // namespace

template <typename T>
void geqrf_panel(Ctx const& c, int64_t m, int64_t n, T* A, int64_t lda, T* tau, T* Tm, int64_t ldt) {
    if (m <= 0 || n <= 0) return;
    int64_t k = std::min(m, n);
    if (!c.dev()) {
        host::geqr2(m, n, A, lda, tau);
        host::larft(m, k, A, lda, tau, Tm, ldt);
        return;
    }
    Scratch sc(c);
    QrPanelDev<T> P;
    P.s = c.stream; P.m = m; P.A0 = A; P.lda = lda; P.tau = tau; P.Tm = Tm; P.ldt = ldt; P.ctx = c;
    int64_t np = ceildiv(m, 256) + 1;
    P.psum = sc.alloc<real_type<T>>(np);
    P.alpha = sc.alloc<T>(2);
    P.pdots = sc.alloc<T>(size_t(np) * 64);
    P.scal = sc.alloc<T>(size_t(k) + 1);
    P.work_elems = int64_t(1) << 20;
    P.work = sc.alloc<T>(P.work_elems);
    P.tsqr_work = sc.alloc<T>(size_t(kd::qr_tsqr_workspace(m)));
    P.ldvp = m;
    P.Vp = sc.alloc<T>(size_t(m) * k);
    // zero all of T (n x n when the panel is wider than tall: the driver's
    // block update multiplies by the full nb x nb T)
    int64_t nt_ = std::min(n, ldt);
    dset(c.stream, 'G', nt_, nt_, T(0), T(0), Tm, ldt);
    P.rec(0, k);
    if (n > k) {
        // wide panel: apply Q^H to the remaining columns
        larfb(c, Side::Left, Op::ConjTrans, m, n - k, k, A, lda, Tm, ldt, A + k * lda, lda);
    }
}

void check_panel_errors() {
    if (!device::available()) return;
    unsigned* w = panel_error_word();
    unsigned h = 0;
    slate_hip_call(hipMemcpy(&h, w, sizeof(h), hipMemcpyDeviceToHost));
    if (h) {
        slate_hip_call(hipMemset(w, 0, sizeof(unsigned)));
        slate_error("persistent panel kernel: a grid-wide hand-off timed out (workgroups not co-resident)");
    }
}

//==============================================================================
// aux
template <typename T>
void set(Ctx const& c, Uplo uplo, int64_t m, int64_t n, T offdiag, T diag, T* A, int64_t lda) {
    if (m <= 0 || n <= 0) return;
    if (!c.dev()) {
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < m; ++i) {
                if (uplo == Uplo::Lower && i < j) continue;
                if (uplo == Uplo::Upper && i > j) continue;
                A[i + j * lda] = i == j ? diag : offdiag;
            }
        return;
    }
    dset(c.stream, upc(uplo), m, n, offdiag, diag, A, lda);
}

template <typename Ts, typename Td>
void copy(Ctx const& c, Uplo uplo, Op op, int64_t m, int64_t n, Ts const* A, int64_t lda, Td* B, int64_t ldb) {
    if (m <= 0 || n <= 0) return;
    if (!c.dev()) {
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < m; ++i) {
                if (uplo == Uplo::Lower && i < j) continue;
                if (uplo == Uplo::Upper && i > j) continue;
                Ts v = host::opval(op, A, lda, i, j);
                if constexpr (is_complex_v<Td>) B[i + j * ldb] = Td(std::real(v), std::imag(v));
                else B[i + j * ldb] = Td(std::real(v));
            }
        return;
    }
    if (std::is_same<Ts, Td>::value && op == Op::NoTrans && uplo == Uplo::General) {
        device::memcpy2d_async(B, ldb * sizeof(Td), A, lda * sizeof(Ts), m * sizeof(Ts), n, c.stream);
        return;
    }
    kd::gecopy(upc(uplo), opc(op), m, n, dptr(A), lda, dptr(B), ldb, c.stream);
}

template <typename T>
void add(Ctx const& c, Uplo uplo, int64_t m, int64_t n, T alpha, T const* A, int64_t lda, T beta, T* B, int64_t ldb) {
    if (m <= 0 || n <= 0) return;
    if (!c.dev()) {
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < m; ++i) {
                if (uplo == Uplo::Lower && i < j) continue;
                if (uplo == Uplo::Upper && i > j) continue;
                B[i + j * ldb] = alpha * A[i + j * lda] + (beta == T(0) ? T(0) : beta * B[i + j * ldb]);
            }
        return;
    }
    kd::geadd(upc(uplo), m, n, dval(alpha), dptr(A), lda, dval(beta), dptr(B), ldb, c.stream);
}

template <typename T>
void scale(Ctx const& c, Uplo uplo, int64_t m, int64_t n, real_type<T> numer, real_type<T> denom, T* A, int64_t lda) {
    if (m <= 0 || n <= 0) return;
    real_type<T> mul = numer / denom;
    if (!c.dev()) {
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < m; ++i) {
                if (uplo == Uplo::Lower && i < j) continue;
                if (uplo == Uplo::Upper && i > j) continue;
                A[i + j * lda] *= mul;
            }
        return;
    }
    kd::gescale(upc(uplo), m, n, mul, dptr(A), lda, c.stream);
}

template <typename T>
void scale_row_col(Ctx const& c, int64_t m, int64_t n, real_type<T> const* R, real_type<T> const* Cs, T* A, int64_t lda) {
    if (m <= 0 || n <= 0) return;
    if (!c.dev()) {
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < m; ++i)
                A[i + j * lda] *= (R ? R[i] : real_type<T>(1)) * (Cs ? Cs[j] : real_type<T>(1));
        return;
    }
    kd::gescale_row_col(m, n, R, Cs, dptr(A), lda, c.stream);
}

template <typename T>
void norm_partial(Ctx const& c, char kind, Uplo uplo, Diag diag, int64_t m, int64_t n, T const* A, int64_t lda,
                  int64_t goff_row, int64_t goff_col, real_type<T>* out) {
    using R = real_type<T>;
    if (m <= 0 || n <= 0) return;
    auto inc = [&](int64_t i, int64_t j) {
        int64_t gi = goff_row + i, gj = goff_col + j;
        return uplo == Uplo::General || (uplo == Uplo::Lower ? gi >= gj : gi <= gj);
    };
    if (!c.dev()) {
        if (kind == 'I') {
            for (int64_t i = 0; i < m; ++i) out[i] = 0;
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = 0; i < m; ++i)
                    if (inc(i, j)) out[i] += (diag == Diag::Unit && goff_row + i == goff_col + j) ? R(1) : std::abs(A[i + j * lda]);
            return;
        }
        for (int64_t j = 0; j < n; ++j) {
            R v = 0, scl = 0, ssq = 1;
            for (int64_t i = 0; i < m; ++i) {
                if (!inc(i, j)) continue;
                R a = (diag == Diag::Unit && goff_row + i == goff_col + j) ? R(1) : std::abs(A[i + j * lda]);
                if (kind == 'M') v = max_nan(v, a);
                else if (kind == '1') v += a;
                else add_sumsq(scl, ssq, a);
            }
            if (kind == 'F') { out[2 * j] = scl; out[2 * j + 1] = scl == 0 ? 0 : ssq; }
            else out[j] = v;
        }
        return;
    }
    Scratch sc(c);
    int64_t cnt = kind == 'I' ? m : (kind == 'F' ? 2 * n : n);
    R* d = sc.alloc<R>(cnt);
    int64_t nw = kd::genorm_work_size(kind, m, n);
    R* w = nw > 0 ? sc.alloc<R>(nw) : nullptr;
    kd::genorm_partial(kind, upc(uplo), char(diag), m, n, dptr(A), lda, goff_row, goff_col, d, c.stream, w);
    device::memcpy_async(out, d, cnt * sizeof(R), c.stream);
    slate_hip_call(hipStreamSynchronize(c.stream));
}

template <typename T>
void copy2d(Ctx const& c, int64_t m, int64_t n, T const* src, int64_t lds, T* dst, int64_t ldd) {
    if (m <= 0 || n <= 0) return;
    if (!c.dev()) {
        for (int64_t j = 0; j < n; ++j) std::memcpy(dst + j * ldd, src + j * lds, m * sizeof(T));
        return;
    }
    device::memcpy2d_async(dst, ldd * sizeof(T), src, lds * sizeof(T), m * sizeof(T), n, c.stream);
}

//==============================================================================
// instantiations
#define SLATE_LB_INST(T)                                                                                   \
    template void gemm<T>(Ctx const&, Op, Op, int64_t, int64_t, int64_t, T, T const*, int64_t, T const*, int64_t, T, T*, int64_t); \
    template void gemm_tri<T>(Ctx const&, Uplo, Op, Op, int64_t, int64_t, T, T const*, int64_t, T const*, int64_t, T, T*, int64_t); \
    template void gemv<T>(Ctx const&, Op, int64_t, int64_t, int64_t, T, T const*, int64_t, T const*, int64_t, T, T*, int64_t); \
    template void gemm_splitk<T>(Ctx const&, Op, Op, int64_t, int64_t, int64_t, int64_t, T, T const*, int64_t, T const*, int64_t, T, T*, int64_t); \
    template void herk<T>(Ctx const&, Uplo, Op, int64_t, int64_t, real_type<T>, T const*, int64_t, real_type<T>, T*, int64_t); \
    template void syrk<T>(Ctx const&, Uplo, Op, int64_t, int64_t, T, T const*, int64_t, T, T*, int64_t);  \
    template void her2k<T>(Ctx const&, Uplo, Op, int64_t, int64_t, T, T const*, int64_t, T const*, int64_t, real_type<T>, T*, int64_t); \
    template void syr2k<T>(Ctx const&, Uplo, Op, int64_t, int64_t, T, T const*, int64_t, T const*, int64_t, T, T*, int64_t); \
    template void hemm<T>(Ctx const&, Side, Uplo, int64_t, int64_t, T, T const*, int64_t, T const*, int64_t, T, T*, int64_t, bool); \
    template void trsm<T>(Ctx const&, Side, Uplo, Op, Diag, int64_t, int64_t, T, T const*, int64_t, T*, int64_t); \
    template void trmm<T>(Ctx const&, Side, Uplo, Op, Diag, int64_t, int64_t, T, T const*, int64_t, T*, int64_t); \
    template void potrf<T>(Ctx const&, Uplo, int64_t, T*, int64_t, int*, int64_t);                        \
    template void trtri<T>(Ctx const&, Uplo, Diag, int64_t, T*, int64_t);                                 \
    template void trtri_to<T>(Ctx const&, Uplo, Diag, int64_t, T const*, int64_t, T*, int64_t);           \
    template void lauum<T>(Ctx const&, Uplo, int64_t, T*, int64_t);                                        \
    template void getrf_panel<T>(Ctx const&, int64_t, int64_t, T*, int64_t, int64_t*, int64_t*, int*, int64_t, bool, bool, double); \
    template void apply_perm<T>(Ctx const&, int64_t, int64_t const*, int64_t const*, int64_t, T*, int64_t); \
    template void geqrf_panel<T>(Ctx const&, int64_t, int64_t, T*, int64_t, T*, T*, int64_t);             \
    template void larfb<T>(Ctx const&, Side, Op, int64_t, int64_t, int64_t, T const*, int64_t, T const*, int64_t, T*, int64_t); \
    template void form_v<T>(Ctx const&, int64_t, int64_t, T const*, int64_t, T*, int64_t);                \
    template void set<T>(Ctx const&, Uplo, int64_t, int64_t, T, T, T*, int64_t);                           \
    template void add<T>(Ctx const&, Uplo, int64_t, int64_t, T, T const*, int64_t, T, T*, int64_t);      \
    template void scale<T>(Ctx const&, Uplo, int64_t, int64_t, real_type<T>, real_type<T>, T*, int64_t);   \
    template void scale_row_col<T>(Ctx const&, int64_t, int64_t, real_type<T> const*, real_type<T> const*, T*, int64_t); \
    template void norm_partial<T>(Ctx const&, char, Uplo, Diag, int64_t, int64_t, T const*, int64_t, int64_t, int64_t, real_type<T>*); \
    template void copy2d<T>(Ctx const&, int64_t, int64_t, T const*, int64_t, T*, int64_t);

SLATE_LB_INST(float)
SLATE_LB_INST(double)
SLATE_LB_INST(std::complex<float>)
SLATE_LB_INST(std::complex<double>)
template void copy2d<int64_t>(Ctx const&, int64_t, int64_t, int64_t const*, int64_t, int64_t*, int64_t);

#define SLATE_LB_COPY(Ts, Td) \
    template void copy<Ts, Td>(Ctx const&, Uplo, Op, int64_t, int64_t, Ts const*, int64_t, Td*, int64_t);
SLATE_LB_COPY(float, float)
SLATE_LB_COPY(double, double)
SLATE_LB_COPY(float, double)
SLATE_LB_COPY(double, float)
SLATE_LB_COPY(std::complex<float>, std::complex<float>)
SLATE_LB_COPY(std::complex<double>, std::complex<double>)
SLATE_LB_COPY(std::complex<float>, std::complex<double>)
SLATE_LB_COPY(std::complex<double>, std::complex<float>)

//------------------------------------------------------------------------------
// Divide-and-conquer merge products (host::stedc_solve) on the GPU.
namespace {
template <typename R>
void stedc_gemm_dev_t(int64_t m, int64_t n, int64_t k, const R* A, int64_t lda, const R* B, int64_t ldb,
                      R* C, int64_t ldc) {
    Ctx c = Ctx::device(device::kTrailQueue);
    device::Buffer<R> dA(size_t(m) * k), dB(size_t(k) * n), dC(size_t(m) * n);
    device::memcpy2d_async(dA.data(), m * sizeof(R), A, lda * sizeof(R), m * sizeof(R), k, c.stream);
    device::memcpy2d_async(dB.data(), k * sizeof(R), B, ldb * sizeof(R), k * sizeof(R), n, c.stream);
    gemm<R>(c, Op::NoTrans, Op::NoTrans, m, n, k, R(1), dA.data(), m, dB.data(), k, R(0), dC.data(), m);
    device::memcpy2d_async(C, ldc * sizeof(R), dC.data(), m * sizeof(R), m * sizeof(R), n, c.stream);
    slate_hip_call(hipStreamSynchronize(c.stream));
}
void stedc_gemm_dev(size_t esize, int64_t m, int64_t n, int64_t k, const void* A, int64_t lda,
                    const void* B, int64_t ldb, void* C, int64_t ldc) {
    if (!device::available()) {
        if (esize == 8) host::gemm<double>(Op::NoTrans, Op::NoTrans, m, n, k, 1.0, (const double*)A, lda,
                                           (const double*)B, ldb, 0.0, (double*)C, ldc);
        else host::gemm<float>(Op::NoTrans, Op::NoTrans, m, n, k, 1.0f, (const float*)A, lda,
                               (const float*)B, ldb, 0.0f, (float*)C, ldc);
        return;
    }
    if (esize == 8) stedc_gemm_dev_t<double>(m, n, k, (const double*)A, lda, (const double*)B, ldb, (double*)C, ldc);
    else stedc_gemm_dev_t<float>(m, n, k, (const float*)A, lda, (const float*)B, ldb, (float*)C, ldc);
}
struct StedcHook { StedcHook() { host::set_stedc_gemm(&stedc_gemm_dev); } } g_stedc_hook;
}  // namespace

}  // namespace lb
}  // namespace slate
