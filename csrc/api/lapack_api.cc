// LAPACK-compatible API (reference lapack_api/, README_lapack_api.txt):
// slate_<p><routine>_ symbols with Fortran calling conventions (every argument
// by reference, trailing hidden string lengths ignored) for
// p in {s, d, c, z}.  Column-major user arrays are wrapped with
// Matrix::fromLAPACK on the 1x1 grid; the computation runs on this process's
// GPU (SLATE_LAPACK_TARGET=d, the default when a GPU is visible) or on the
// host (=h), with tile size SLATE_LAPACK_NB (default 512 on the GPU, 256 on
// the host).  Results are copied back to the user's arrays before returning.
//
// Intra-process multi-GPU (reference lapack_api/lapack_slate.hh: the shim
// goes to the device target whenever GPUs exist, and its rank spreads tiles
// over all of them): when inproc_ranks() > 1 -- every visible GPU by default,
// or $SLATE_INPROC_RANKS -- the factorizations / solves / gemm below run on a
// p x q grid of in-process ranks, one per GPU (inproc.hh), each copying its
// own tiles in from and back out to the caller's array.
#include "slate_amd/slate.hh"
#include "slate_amd/device.hh"
#include "slate_amd/inproc.hh"

#include <cctype>
#include <complex>
#include <cstdlib>
#include <cstring>

namespace {

using namespace slate;

Target lapack_target() {
    const char* e = std::getenv("SLATE_LAPACK_TARGET");
    if (e && (std::tolower(e[0]) == 'h' || std::tolower(e[0]) == 't')) return Target::Host;
    if (e && std::tolower(e[0]) == 'd') return Target::Devices;
    return device::available() ? Target::Devices : Target::Host;
}

int64_t lapack_nb(Target t) {
    if (const char* e = std::getenv("SLATE_LAPACK_NB")) return std::max(1, std::atoi(e));
    return t == Target::Devices ? 512 : 256;
}

Options lapack_opts() { return {{Option::Target, lapack_target()}, {Option::Lookahead, int64_t(1)}}; }

inline char up(char const* c) { return char(std::toupper(*c)); }
inline Op op_of(char const* c) { char t = up(c); return t == 'N' ? Op::NoTrans : t == 'T' ? Op::Trans : Op::ConjTrans; }
inline Uplo uplo_of(char const* c) { return up(c) == 'U' ? Uplo::Upper : Uplo::Lower; }
inline Diag diag_of(char const* c) { return up(c) == 'U' ? Diag::Unit : Diag::NonUnit; }
inline Side side_of(char const* c) { return up(c) == 'L' ? Side::Left : Side::Right; }
inline Norm norm_of(char const* c) {
    char t = up(c);
    if (t == '1' || t == 'O') return Norm::One;
    if (t == 'I') return Norm::Inf;
    if (t == 'F' || t == 'E') return Norm::Fro;
    return Norm::Max;
}

template <typename T>
Matrix<T> wrap(int64_t m, int64_t n, T* A, int64_t lda, Target t) {
    Matrix<T> M = Matrix<T>::fromLAPACK(m, n, A, lda, lapack_nb(t));
    if (t == Target::Devices) M.insertLocalTiles(Target::Devices);
    return M;
}

template <typename T>
void done(BaseMatrix<T>& A) { A.tileUpdateAllOrigin(); }

/// One caller array of an in-process multi-rank call.
struct HostArg { void* A; int64_t m, n, ld; bool out; };

/// Run body(mats, rank) on the in-process grid with each array distributed
/// (2-D block cyclic, tile size lapack_nb) when more than one rank is
/// configured and the problem has at least as many tile rows as ranks;
/// returns false (caller takes the one-rank path) otherwise.
template <typename T>
bool run_multi(std::vector<HostArg> const& args, std::function<void(std::vector<Matrix<T>>&, int)> const& body) {
    const int nr = inproc_ranks();
    if (nr <= 1 || args.empty()) return false;
    const Target t = lapack_target();
    const int64_t nb = lapack_nb(t);
    if ((args[0].m + nb - 1) / nb < 2) return false;   // too small to split
    int p, q;
    inproc_grid_shape(nr, p, q);
    run_in_process(p, q, [&](int rank, GridPtr const& g) {
        std::vector<Matrix<T>> M;
        for (auto const& a : args) {
            Matrix<T> X(a.m, a.n, nb, g);
            X.insertLocalTiles(t);
            scatter_from_host(static_cast<T const*>(a.A), a.ld, X, t);
            M.push_back(X);
        }
        body(M, rank);
        for (size_t i = 0; i < args.size(); ++i)
            if (args[i].out) gather_to_host(M[i], static_cast<T*>(args[i].A), args[i].ld);
    });
    return true;
}

// LAPACK ipiv (1-based global rows) <-> Pivots (tile offset, element offset)
template <typename T>
void to_ipiv(Matrix<T> const& A, Pivots const& P, int* ipiv) {
    const int64_t nb = A.nb();
    int64_t r = 0;
    for (int64_t k = 0; k < int64_t(P.size()); ++k)
        for (auto const& p : P[k]) ipiv[r++] = int((k + p.tileIndex()) * nb + p.elementOffset() + 1);
}

template <typename T>
Pivots from_ipiv(Matrix<T> const& A, int64_t kmin, int const* ipiv) {
    const int64_t nb = A.nb();
    Pivots P((kmin + nb - 1) / nb);
    for (int64_t j = 0; j < kmin; ++j) {
        int64_t k = j / nb, row = ipiv[j] - 1;
        P[k].push_back(Pivot(row / nb - k, row % nb));
    }
    return P;
}

//------------------------------------------------------------------------------
template <typename T>
void gemm_(char const* ta, char const* tb, int const* m, int const* n, int const* k, T const* alpha, T* A,
           int const* lda, T* B, int const* ldb, T const* beta, T* C, int const* ldc) {
    Target t = lapack_target();
    Op oa = op_of(ta), ob = op_of(tb);
    const int64_t am = oa == Op::NoTrans ? *m : *k, an = oa == Op::NoTrans ? *k : *m;
    const int64_t bm = ob == Op::NoTrans ? *k : *n, bn = ob == Op::NoTrans ? *n : *k;
    if (run_multi<T>({{C, *m, *n, *ldc, true}, {A, am, an, *lda, false}, {B, bm, bn, *ldb, false}},
                     [&](std::vector<Matrix<T>>& M, int) {
                         Matrix<T> Ao = oa == Op::NoTrans ? M[1] : oa == Op::Trans ? transpose(M[1]) : conj_transpose(M[1]);
                         Matrix<T> Bo = ob == Op::NoTrans ? M[2] : ob == Op::Trans ? transpose(M[2]) : conj_transpose(M[2]);
                         gemm(*alpha, Ao, Bo, *beta, M[0], lapack_opts());
                     }))
        return;
    auto Am = wrap(oa == Op::NoTrans ? *m : *k, oa == Op::NoTrans ? *k : *m, A, *lda, t);
    auto Bm = wrap(ob == Op::NoTrans ? *k : *n, ob == Op::NoTrans ? *n : *k, B, *ldb, t);
    auto Cm = wrap<T>(*m, *n, C, *ldc, t);
    Matrix<T> Ao = oa == Op::NoTrans ? Am : oa == Op::Trans ? transpose(Am) : conj_transpose(Am);
    Matrix<T> Bo = ob == Op::NoTrans ? Bm : ob == Op::Trans ? transpose(Bm) : conj_transpose(Bm);
    gemm(*alpha, Ao, Bo, *beta, Cm, lapack_opts());
    done(Cm);
}

template <typename T>
void hemm_(bool herm, char const* side, char const* uplo, int const* m, int const* n, T const* alpha, T* A,
           int const* lda, T* B, int const* ldb, T const* beta, T* C, int const* ldc) {
    Target t = lapack_target();
    int64_t na = side_of(side) == Side::Left ? *m : *n;
    auto Am = wrap<T>(na, na, A, *lda, t);
    auto Bm = wrap<T>(*m, *n, B, *ldb, t);
    auto Cm = wrap<T>(*m, *n, C, *ldc, t);
    if (herm) hemm(side_of(side), *alpha, HermitianMatrix<T>(uplo_of(uplo), Am), Bm, *beta, Cm, lapack_opts());
    else symm(side_of(side), *alpha, SymmetricMatrix<T>(uplo_of(uplo), Am), Bm, *beta, Cm, lapack_opts());
    done(Cm);
}

template <typename T>
void herk_(bool herm, char const* uplo, char const* trans, int const* n, int const* k, T const* alpha, T* A,
           int const* lda, T const* beta, T* C, int const* ldc) {
    Target t = lapack_target();
    Op o = op_of(trans);
    auto Am = wrap<T>(o == Op::NoTrans ? *n : *k, o == Op::NoTrans ? *k : *n, A, *lda, t);
    Matrix<T> Ao = o == Op::NoTrans ? Am : (herm ? conj_transpose(Am) : transpose(Am));
    auto Cm = wrap<T>(*n, *n, C, *ldc, t);
    if (herm) {
        HermitianMatrix<T> H(uplo_of(uplo), Cm);
        herk(std::real(*alpha), Ao, std::real(*beta), H, lapack_opts());
    } else {
        SymmetricMatrix<T> S(uplo_of(uplo), Cm);
        syrk(*alpha, Ao, *beta, S, lapack_opts());
    }
    done(Cm);
}

template <typename T>
void her2k_(bool herm, char const* uplo, char const* trans, int const* n, int const* k, T const* alpha, T* A,
            int const* lda, T* B, int const* ldb, T const* beta, T* C, int const* ldc) {
    Target t = lapack_target();
    Op o = op_of(trans);
    int64_t r = o == Op::NoTrans ? *n : *k, c = o == Op::NoTrans ? *k : *n;
    auto Am = wrap<T>(r, c, A, *lda, t);
    auto Bm = wrap<T>(r, c, B, *ldb, t);
    Matrix<T> Ao = o == Op::NoTrans ? Am : (herm ? conj_transpose(Am) : transpose(Am));
    Matrix<T> Bo = o == Op::NoTrans ? Bm : (herm ? conj_transpose(Bm) : transpose(Bm));
    auto Cm = wrap<T>(*n, *n, C, *ldc, t);
    if (herm) {
        HermitianMatrix<T> H(uplo_of(uplo), Cm);
        her2k(*alpha, Ao, Bo, std::real(*beta), H, lapack_opts());
    } else {
        SymmetricMatrix<T> S(uplo_of(uplo), Cm);
        syr2k(*alpha, Ao, Bo, *beta, S, lapack_opts());
    }
    done(Cm);
}

template <typename T>
void trmm_(bool solve, char const* side, char const* uplo, char const* transa, char const* diag, int const* m,
           int const* n, T const* alpha, T* A, int const* lda, T* B, int const* ldb) {
    Target t = lapack_target();
    int64_t na = side_of(side) == Side::Left ? *m : *n;
    auto Am = wrap<T>(na, na, A, *lda, t);
    auto Bm = wrap<T>(*m, *n, B, *ldb, t);
    TriangularMatrix<T> Tm(uplo_of(uplo), diag_of(diag), Am);
    Op o = op_of(transa);
    TriangularMatrix<T> To = o == Op::NoTrans ? Tm : o == Op::Trans ? transpose(Tm) : conj_transpose(Tm);
    if (solve) trsm(side_of(side), *alpha, To, Bm, lapack_opts());
    else trmm(side_of(side), *alpha, To, Bm, lapack_opts());
    done(Bm);
}

template <typename T>
void getrf_(int const* m, int const* n, T* A, int const* lda, int* ipiv, int* info) {
    if (run_multi<T>({{A, *m, *n, *lda, true}}, [&](std::vector<Matrix<T>>& M, int rank) {
            Pivots P;
            int inf = int(getrf(M[0], P, lapack_opts()));
            if (rank == 0) { *info = inf; to_ipiv(M[0], P, ipiv); }
        }))
        return;
    Target t = lapack_target();
    auto Am = wrap<T>(*m, *n, A, *lda, t);
    Pivots P;
    *info = int(getrf(Am, P, lapack_opts()));
    done(Am);
    to_ipiv(Am, P, ipiv);
}

template <typename T>
void getrs_(char const* trans, int const* n, int const* nrhs, T* A, int const* lda, int const* ipiv, T* B,
            int const* ldb, int* info) {
    *info = 0;
    if (run_multi<T>({{A, *n, *n, *lda, false}, {B, *n, *nrhs, *ldb, true}}, [&](std::vector<Matrix<T>>& M, int) {
            Pivots P = from_ipiv(M[0], *n, ipiv);
            getrs(op_of(trans), M[0], P, M[1], lapack_opts());
        }))
        return;
    Target t = lapack_target();
    auto Am = wrap<T>(*n, *n, A, *lda, t);
    auto Bm = wrap<T>(*n, *nrhs, B, *ldb, t);
    Pivots P = from_ipiv(Am, *n, ipiv);
    getrs(op_of(trans), Am, P, Bm, lapack_opts());
    done(Bm);
    *info = 0;
}

template <typename T>
void gesv_(int const* n, int const* nrhs, T* A, int const* lda, int* ipiv, T* B, int const* ldb, int* info) {
    if (run_multi<T>({{A, *n, *n, *lda, true}, {B, *n, *nrhs, *ldb, true}}, [&](std::vector<Matrix<T>>& M, int rank) {
            Pivots P;
            int inf = int(gesv(M[0], P, M[1], lapack_opts()));
            if (rank == 0) { *info = inf; to_ipiv(M[0], P, ipiv); }
        }))
        return;
    Target t = lapack_target();
    auto Am = wrap<T>(*n, *n, A, *lda, t);
    auto Bm = wrap<T>(*n, *nrhs, B, *ldb, t);
    Pivots P;
    *info = int(gesv(Am, P, Bm, lapack_opts()));
    done(Am);
    done(Bm);
    to_ipiv(Am, P, ipiv);
}

template <typename T>
void gesv_mixed_(int const* n, int const* nrhs, T* A, int const* lda, int* ipiv, T* B, int const* ldb, T* X,
                 int const* ldx, int* iter, int* info) {
    Target t = lapack_target();
    auto Am = wrap<T>(*n, *n, A, *lda, t);
    auto Bm = wrap<T>(*n, *nrhs, B, *ldb, t);
    auto Xm = wrap<T>(*n, *nrhs, X, *ldx, t);
    Pivots P;
    int it = 0;
    *info = int(gesv_mixed(Am, P, Bm, Xm, it, lapack_opts()));
    *iter = it;
    done(Am);
    done(Xm);
    if (!P.empty()) to_ipiv(Am, P, ipiv);
}

template <typename T>
void getri_(int const* n, T* A, int const* lda, int const* ipiv, int* info) {
    Target t = lapack_target();
    auto Am = wrap<T>(*n, *n, A, *lda, t);
    Pivots P = from_ipiv(Am, *n, ipiv);
    *info = int(getri(Am, P, lapack_opts()));
    done(Am);
}

template <typename T>
void potrf_(char const* uplo, int const* n, T* A, int const* lda, int* info) {
    if (run_multi<T>({{A, *n, *n, *lda, true}}, [&](std::vector<Matrix<T>>& M, int rank) {
            HermitianMatrix<T> H(uplo_of(uplo), M[0]);
            int inf = int(potrf(H, lapack_opts()));
            if (rank == 0) *info = inf;
        }))
        return;
    Target t = lapack_target();
    auto Am = wrap<T>(*n, *n, A, *lda, t);
    HermitianMatrix<T> H(uplo_of(uplo), Am);
    *info = int(potrf(H, lapack_opts()));
    done(Am);
}

template <typename T>
void posv_(char const* uplo, int const* n, int const* nrhs, T* A, int const* lda, T* B, int const* ldb, int* info) {
    if (run_multi<T>({{A, *n, *n, *lda, true}, {B, *n, *nrhs, *ldb, true}}, [&](std::vector<Matrix<T>>& M, int rank) {
            HermitianMatrix<T> H(uplo_of(uplo), M[0]);
            int inf = int(posv(H, M[1], lapack_opts()));
            if (rank == 0) *info = inf;
        }))
        return;
    Target t = lapack_target();
    auto Am = wrap<T>(*n, *n, A, *lda, t);
    auto Bm = wrap<T>(*n, *nrhs, B, *ldb, t);
    HermitianMatrix<T> H(uplo_of(uplo), Am);
    *info = int(posv(H, Bm, lapack_opts()));
    done(Am);
    done(Bm);
}

template <typename T>
void potri_(char const* uplo, int const* n, T* A, int const* lda, int* info) {
    Target t = lapack_target();
    auto Am = wrap<T>(*n, *n, A, *lda, t);
    HermitianMatrix<T> H(uplo_of(uplo), Am);
    *info = int(potri(H, lapack_opts()));
    done(Am);
}

template <typename T>
void gels_(char const* trans, int const* m, int const* n, int const* nrhs, T* A, int const* lda, T* B,
           int const* ldb, int* info) {
    Target t = lapack_target();
    *info = 0;
    if (op_of(trans) != Op::NoTrans) { *info = -1; return; }
    auto Am = wrap<T>(*m, *n, A, *lda, t);
    auto Bm = wrap<T>(std::max(*m, *n), *nrhs, B, *ldb, t);
    TriangularFactors<T> Tf;
    gels(Am, Tf, Bm, lapack_opts());
    done(Am);
    done(Bm);
}

template <typename T>
void gecon_(char const* norm, int const* n, T* A, int const* lda, real_type<T> const* anorm,
            real_type<T>* rcond, int* info) {
    Target t = lapack_target();
    auto Am = wrap<T>(*n, *n, A, *lda, t);
    *rcond = gecondest(norm_of(norm), Am, *anorm, lapack_opts());
    *info = 0;
}

template <typename T>
void pocon_(char const* uplo, int const* n, T* A, int const* lda, real_type<T> const* anorm, real_type<T>* rcond,
            int* info) {
    Target t = lapack_target();
    auto Am = wrap<T>(*n, *n, A, *lda, t);
    HermitianMatrix<T> H(uplo_of(uplo), Am);
    *rcond = pocondest(Norm::One, H, *anorm, lapack_opts());
    *info = 0;
}

template <typename T>
void trcon_(char const* norm, char const* uplo, char const* diag, int const* n, T* A, int const* lda,
            real_type<T>* rcond, int* info) {
    Target t = lapack_target();
    auto Am = wrap<T>(*n, *n, A, *lda, t);
    TriangularMatrix<T> Tm(uplo_of(uplo), diag_of(diag), Am);
    *rcond = trcondest(norm_of(norm), Tm, lapack_opts());
    *info = 0;
}

template <typename T>
real_type<T> lange_(char const* norm, int const* m, int const* n, T* A, int const* lda) {
    Target t = lapack_target();
    auto Am = wrap<T>(*m, *n, A, *lda, t);
    return slate::norm(norm_of(norm), Am, lapack_opts());
}

template <typename T>
real_type<T> lanhe_(bool herm, char const* norm, char const* uplo, int const* n, T* A, int const* lda) {
    Target t = lapack_target();
    auto Am = wrap<T>(*n, *n, A, *lda, t);
    if (herm) return slate::norm(norm_of(norm), HermitianMatrix<T>(uplo_of(uplo), Am), lapack_opts());
    return slate::norm(norm_of(norm), SymmetricMatrix<T>(uplo_of(uplo), Am), lapack_opts());
}

template <typename T>
real_type<T> lantr_(char const* norm, char const* uplo, char const* diag, int const* m, int const* n, T* A,
                    int const* lda) {
    Target t = lapack_target();
    auto Am = wrap<T>(*m, *n, A, *lda, t);
    return slate::norm(norm_of(norm), TrapezoidMatrix<T>(uplo_of(uplo), diag_of(diag), Am), lapack_opts());
}

template <typename T>
void heev_(char const* jobz, char const* uplo, int const* n, T* A, int const* lda, real_type<T>* W, int* info) {
    Target t = lapack_target();
    auto Am = wrap<T>(*n, *n, A, *lda, t);
    HermitianMatrix<T> H(uplo_of(uplo), Am);
    std::vector<real_type<T>> L;
    Matrix<T> Z;
    bool vec = up(jobz) == 'V';
    if (vec) { Z = Am.emptyLike(); Z.insertLocalTiles(t); }
    heev(H, L, Z, lapack_opts());
    std::copy(L.begin(), L.end(), W);
    if (vec) { slate::copy<T, T>(Z, Am, lapack_opts()); done(Am); }
    *info = 0;
}

template <typename T>
void gesvd_(char const* jobu, char const* jobvt, int const* m, int const* n, T* A, int const* lda,
            real_type<T>* S, T* U, int const* ldu, T* VT, int const* ldvt, int* info) {
    Target t = lapack_target();
    *info = 0;
    const int64_t k = std::min(*m, *n);
    char ju = up(jobu), jv = up(jobvt);
    if ((ju == 'A' && *m != k) || (jv == 'A' && *n != k) || ju == 'O' || jv == 'O') { *info = -1; return; }
    auto Am = wrap<T>(*m, *n, A, *lda, t);
    Matrix<T> Um, Vm;
    if (ju != 'N') Um = wrap<T>(*m, k, U, *ldu, t);
    if (jv != 'N') Vm = wrap<T>(k, *n, VT, *ldvt, t);
    std::vector<real_type<T>> Sv;
    svd(Am, Sv, Um, Vm, lapack_opts());
    std::copy(Sv.begin(), Sv.end(), S);
    if (ju != 'N') done(Um);
    if (jv != 'N') done(Vm);
}

}  // namespace

//------------------------------------------------------------------------------
// Fortran-callable symbols (lowercase + underscore, as the reference exports)
#define SLATE_LAPACK_API(p, T)                                                                             \
extern "C" {                                                                                               \
void slate_##p##gemm_(char const* ta, char const* tb, int const* m, int const* n, int const* k, T const* al, \
                      T* A, int const* lda, T* B, int const* ldb, T const* be, T* C, int const* ldc) {    \
    gemm_<T>(ta, tb, m, n, k, al, A, lda, B, ldb, be, C, ldc); }                                           \
void slate_##p##symm_(char const* sd, char const* ul, int const* m, int const* n, T const* al, T* A,      \
                      int const* lda, T* B, int const* ldb, T const* be, T* C, int const* ldc) {          \
    hemm_<T>(false, sd, ul, m, n, al, A, lda, B, ldb, be, C, ldc); }                                       \
void slate_##p##syrk_(char const* ul, char const* tr, int const* n, int const* k, T const* al, T* A,      \
                      int const* lda, T const* be, T* C, int const* ldc) {                                \
    herk_<T>(false, ul, tr, n, k, al, A, lda, be, C, ldc); }                                               \
void slate_##p##syr2k_(char const* ul, char const* tr, int const* n, int const* k, T const* al, T* A,     \
                       int const* lda, T* B, int const* ldb, T const* be, T* C, int const* ldc) {         \
    her2k_<T>(false, ul, tr, n, k, al, A, lda, B, ldb, be, C, ldc); }                                      \
void slate_##p##trmm_(char const* sd, char const* ul, char const* ta, char const* dg, int const* m,        \
                      int const* n, T const* al, T* A, int const* lda, T* B, int const* ldb) {            \
    trmm_<T>(false, sd, ul, ta, dg, m, n, al, A, lda, B, ldb); }                                           \
void slate_##p##trsm_(char const* sd, char const* ul, char const* ta, char const* dg, int const* m,        \
                      int const* n, T const* al, T* A, int const* lda, T* B, int const* ldb) {            \
    trmm_<T>(true, sd, ul, ta, dg, m, n, al, A, lda, B, ldb); }                                            \
void slate_##p##getrf_(int const* m, int const* n, T* A, int const* lda, int* ipiv, int* info) {          \
    getrf_<T>(m, n, A, lda, ipiv, info); }                                                                 \
void slate_##p##getrs_(char const* tr, int const* n, int const* nrhs, T* A, int const* lda, int const* ipiv, \
                       T* B, int const* ldb, int* info) {                                                  \
    getrs_<T>(tr, n, nrhs, A, lda, ipiv, B, ldb, info); }                                                  \
void slate_##p##gesv_(int const* n, int const* nrhs, T* A, int const* lda, int* ipiv, T* B, int const* ldb, \
                      int* info) {                                                                         \
    gesv_<T>(n, nrhs, A, lda, ipiv, B, ldb, info); }                                                       \
void slate_##p##getri_(int const* n, T* A, int const* lda, int const* ipiv, T*, int const*, int* info) {  \
    getri_<T>(n, A, lda, ipiv, info); }                                                                    \
void slate_##p##potrf_(char const* ul, int const* n, T* A, int const* lda, int* info) {                  \
    potrf_<T>(ul, n, A, lda, info); }                                                                      \
void slate_##p##posv_(char const* ul, int const* n, int const* nrhs, T* A, int const* lda, T* B,         \
                      int const* ldb, int* info) {                                                         \
    posv_<T>(ul, n, nrhs, A, lda, B, ldb, info); }                                                         \
void slate_##p##potri_(char const* ul, int const* n, T* A, int const* lda, int* info) {                  \
    potri_<T>(ul, n, A, lda, info); }                                                                      \
void slate_##p##gels_(char const* tr, int const* m, int const* n, int const* nrhs, T* A, int const* lda,  \
                      T* B, int const* ldb, T*, int const*, int* info) {                                   \
    gels_<T>(tr, m, n, nrhs, A, lda, B, ldb, info); }                                                      \
void slate_##p##gecon_(char const* nm, int const* n, T* A, int const* lda, real_type<T> const* an,        \
                       real_type<T>* rc, T*, void*, int* info) {                                           \
    gecon_<T>(nm, n, A, lda, an, rc, info); }                                                              \
void slate_##p##pocon_(char const* ul, int const* n, T* A, int const* lda, real_type<T> const* an,        \
                       real_type<T>* rc, T*, void*, int* info) {                                           \
    pocon_<T>(ul, n, A, lda, an, rc, info); }                                                              \
void slate_##p##trcon_(char const* nm, char const* ul, char const* dg, int const* n, T* A, int const* lda, \
                       real_type<T>* rc, T*, void*, int* info) {                                           \
    trcon_<T>(nm, ul, dg, n, A, lda, rc, info); }                                                          \
real_type<T> slate_##p##lange_(char const* nm, int const* m, int const* n, T* A, int const* lda,         \
                               real_type<T>*) {                                                            \
    return lange_<T>(nm, m, n, A, lda); }                                                                  \
real_type<T> slate_##p##lansy_(char const* nm, char const* ul, int const* n, T* A, int const* lda,       \
                               real_type<T>*) {                                                            \
    return lanhe_<T>(false, nm, ul, n, A, lda); }                                                          \
real_type<T> slate_##p##lantr_(char const* nm, char const* ul, char const* dg, int const* m, int const* n, \
                               T* A, int const* lda, real_type<T>*) {                                      \
    return lantr_<T>(nm, ul, dg, m, n, A, lda); }                                                          \
void slate_##p##gesvd_(char const* ju, char const* jv, int const* m, int const* n, T* A, int const* lda,  \
                       real_type<T>* S, T* U, int const* ldu, T* VT, int const* ldvt, T*, int const*,     \
                       int* info) {                                                                        \
    gesvd_<T>(ju, jv, m, n, A, lda, S, U, ldu, VT, ldvt, info); }                                          \
}

#define SLATE_LAPACK_API_REAL(p, T)                                                                        \
extern "C" {                                                                                               \
void slate_##p##syev_(char const* jz, char const* ul, int const* n, T* A, int const* lda, T* W, T*,       \
                      int const*, int* info) { heev_<T>(jz, ul, n, A, lda, W, info); }                     \
void slate_##p##syevd_(char const* jz, char const* ul, int const* n, T* A, int const* lda, T* W, T*,      \
                       int const*, int*, int const*, int* info) { heev_<T>(jz, ul, n, A, lda, W, info); }  \
}

#define SLATE_LAPACK_API_CPLX(p, T)                                                                        \
extern "C" {                                                                                               \
void slate_##p##hemm_(char const* sd, char const* ul, int const* m, int const* n, T const* al, T* A,      \
                      int const* lda, T* B, int const* ldb, T const* be, T* C, int const* ldc) {          \
    hemm_<T>(true, sd, ul, m, n, al, A, lda, B, ldb, be, C, ldc); }                                        \
void slate_##p##herk_(char const* ul, char const* tr, int const* n, int const* k, real_type<T> const* al, \
                      T* A, int const* lda, real_type<T> const* be, T* C, int const* ldc) {               \
    T a(*al), b(*be); herk_<T>(true, ul, tr, n, k, &a, A, lda, &b, C, ldc); }                              \
void slate_##p##her2k_(char const* ul, char const* tr, int const* n, int const* k, T const* al, T* A,     \
                       int const* lda, T* B, int const* ldb, real_type<T> const* be, T* C, int const* ldc) { \
    T b(*be); her2k_<T>(true, ul, tr, n, k, al, A, lda, B, ldb, &b, C, ldc); }                             \
real_type<T> slate_##p##lanhe_(char const* nm, char const* ul, int const* n, T* A, int const* lda,       \
                               real_type<T>*) {                                                            \
    return lanhe_<T>(true, nm, ul, n, A, lda); }                                                           \
void slate_##p##heev_(char const* jz, char const* ul, int const* n, T* A, int const* lda, real_type<T>* W, \
                      T*, int const*, real_type<T>*, int* info) { heev_<T>(jz, ul, n, A, lda, W, info); } \
void slate_##p##heevd_(char const* jz, char const* ul, int const* n, T* A, int const* lda,                 \
                       real_type<T>* W, T*, int const*, real_type<T>*, int const*, int*, int const*,       \
                       int* info) { heev_<T>(jz, ul, n, A, lda, W, info); }                                \
}

SLATE_LAPACK_API(s, float)
SLATE_LAPACK_API(d, double)
SLATE_LAPACK_API(c, std::complex<float>)
SLATE_LAPACK_API(z, std::complex<double>)
SLATE_LAPACK_API_REAL(s, float)
SLATE_LAPACK_API_REAL(d, double)
SLATE_LAPACK_API_CPLX(c, std::complex<float>)
SLATE_LAPACK_API_CPLX(z, std::complex<double>)

extern "C" {
/// LAPACK dsgesv / zcgesv: fp32 factorization + fp64 refinement.
void slate_dsgesv_(int const* n, int const* nrhs, double* A, int const* lda, int* ipiv, double* B, int const* ldb,
                   double* X, int const* ldx, double*, float*, int* iter, int* info) {
    gesv_mixed_<double>(n, nrhs, A, lda, ipiv, B, ldb, X, ldx, iter, info);
}
void slate_zcgesv_(int const* n, int const* nrhs, std::complex<double>* A, int const* lda, int* ipiv,
                   std::complex<double>* B, int const* ldb, std::complex<double>* X, int const* ldx,
                   std::complex<double>*, std::complex<float>*, double*, int* iter, int* info) {
    gesv_mixed_<std::complex<double>>(n, nrhs, A, lda, ipiv, B, ldb, X, ldx, iter, info);
}
}
