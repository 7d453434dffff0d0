// ScaLAPACK-compatible API (reference scalapack_api/, README_scalapack_api.txt):
// p<p><routine>_ symbols (plus UPPERCASE and no-underscore aliases) taking
// ScaLAPACK array descriptors desc[9] = {dtype, ctxt, M, N, MB, NB, RSRC,
// CSRC, LLD}.  The local arrays are wrapped in place with
// Matrix::fromScaLAPACK on the process grid installed by the framework
// (slate_d35_amd.parallel.init_grid / set_default_grid), whose p x q must match
// the BLACS context's; the descriptor's ctxt is not interpreted (there is no
// BLACS in this stack).  Sub-matrices A(IA:, JA:) must start on a tile
// boundary, as in the reference.  Target / lookahead come from
// SLATE_SCALAPACK_TARGET (d|h) and SLATE_SCALAPACK_LOOKAHEAD.
#include "slate_amd/slate.hh"
#include "slate_amd/device.hh"

#include <cctype>
#include <complex>
#include <cstdlib>

namespace {

using namespace slate;

enum { DTYPE_ = 0, CTXT_, M_, N_, MB_, NB_, RSRC_, CSRC_, LLD_ };

Target sl_target() {
    const char* e = std::getenv("SLATE_SCALAPACK_TARGET");
    if (e && std::tolower(e[0]) == 'h') return Target::Host;
    if (e && std::tolower(e[0]) == 'd') return Target::Devices;
    return device::available() ? Target::Devices : Target::Host;
}

Options sl_opts() {
    int64_t la = 1;
    if (const char* e = std::getenv("SLATE_SCALAPACK_LOOKAHEAD")) la = std::atoi(e);
    return {{Option::Target, sl_target()}, {Option::Lookahead, la}};
}

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

/// The m x n sub-matrix A(ia:ia+m-1, ja:ja+n-1) of the distributed array.
template <typename T>
Matrix<T> wrap(int64_t m, int64_t n, T* A, int const* ia, int const* ja, int const* desc) {
    Target t = sl_target();
    const int64_t mb = desc[MB_], nb = desc[NB_];
    slate_error_if_msg((*ia - 1) % mb != 0 || (*ja - 1) % nb != 0,
                       "ScaLAPACK API: sub-matrix must start on a tile boundary");
    Matrix<T> G = Matrix<T>::fromScaLAPACK(desc[M_], desc[N_], A, desc[LLD_], mb, nb, default_grid(), Loc::Host,
                                           desc[RSRC_], desc[CSRC_]);
    if (t == Target::Devices) G.insertLocalTiles(Target::Devices);
    int64_t i1 = (*ia - 1) / mb, j1 = (*ja - 1) / nb;
    int64_t i2 = m > 0 ? (*ia - 1 + m - 1) / mb : i1 - 1, j2 = n > 0 ? (*ja - 1 + n - 1) / nb : j1 - 1;
    Matrix<T> S = G.sub(i1, i2, j1, j2);
    if (S.m() != m || S.n() != n) S = G.slice(*ia - 1, *ia - 1 + m - 1, *ja - 1, *ja - 1 + n - 1);
    return S;
}

template <typename T>
void done(BaseMatrix<T>& A) { A.tileUpdateAllOrigin(); }

template <typename T>
void to_ipiv(Matrix<T> const& A, Pivots const& P, int* ipiv) {
    // local ipiv (ScaLAPACK): one entry per local row of the tile rows I own
    // in A's column; here every rank receives all pivots of the factored
    // column range (global row indices, 1-based) and stores its local slice.
    const int64_t nb = A.nb();
    std::vector<int> all;
    for (int64_t k = 0; k < int64_t(P.size()); ++k)
        for (auto const& p : P[k]) all.push_back(int((k + p.tileIndex()) * nb + p.elementOffset() + 1));
    auto& g = *A.grid();
    int64_t r = 0;
    for (int64_t i = 0; i < A.mt(); ++i) {
        if (A.srow_owner(i) != g.myrow()) continue;
        for (int64_t t = 0; t < A.tileMb(i); ++t) {
            int64_t gi = i * nb + t;
            ipiv[r++] = gi < int64_t(all.size()) ? all[gi] : int(gi + 1);
        }
    }
}

template <typename T>
Pivots from_ipiv(Matrix<T> const& A, int64_t kmin, int const* ipiv) {
    // gather the global pivot vector from the local slices (sum-allreduce)
    const int64_t nb = A.nb();
    auto& g = *A.grid();
    std::vector<int64_t> all(kmin, 0);
    int64_t r = 0;
    for (int64_t i = 0; i < A.mt(); ++i) {
        if (A.srow_owner(i) != g.myrow()) continue;
        for (int64_t t = 0; t < A.tileMb(i); ++t, ++r) {
            int64_t gi = i * nb + t;
            if (gi < kmin && g.mycol() == 0) all[gi] = ipiv[r];
        }
    }
    if (g.size() > 1) g.world().allreduce(all.data(), all.data(), all.size(), ScalarType::Int64, ReduceOp::Sum,
                                          Loc::Host, nullptr);
    Pivots P((kmin + nb - 1) / nb);
    for (int64_t j = 0; j < kmin; ++j) {
        int64_t k = j / nb, row = all[j] - 1;
        P[k].push_back(Pivot(row / nb - k, row % nb));
    }
    return P;
}

#define SUB(X, m, n) wrap<T>(m, n, X, i##X, j##X, desc##X)

template <typename T>
void pgemm(char const* ta, char const* tb, int const* m, int const* n, int const* k, T const* alpha, T* A,
           int const* iA, int const* jA, int const* descA, T* B, int const* iB, int const* jB, int const* descB,
           T const* beta, T* C, int const* iC, int const* jC, int const* descC) {
    Op oa = op_of(ta), ob = op_of(tb);
    auto Am = SUB(A, oa == Op::NoTrans ? *m : *k, oa == Op::NoTrans ? *k : *m);
    auto Bm = SUB(B, ob == Op::NoTrans ? *k : *n, ob == Op::NoTrans ? *n : *k);
    auto Cm = SUB(C, *m, *n);
    Matrix<T> Ao = oa == Op::NoTrans ? Am : oa == Op::Trans ? transpose(Am) : conj_transpose(Am);
    Matrix<T> Bo = ob == Op::NoTrans ? Bm : ob == Op::Trans ? transpose(Bm) : conj_transpose(Bm);
    gemm(*alpha, Ao, Bo, *beta, Cm, sl_opts());
    done(Cm);
}

template <typename T>
void phemm(bool herm, char const* side, char const* uplo, int const* m, int const* n, T const* alpha, T* A,
           int const* iA, int const* jA, int const* descA, T* B, int const* iB, int const* jB, int const* descB,
           T const* beta, T* C, int const* iC, int const* jC, int const* descC) {
    int64_t na = side_of(side) == Side::Left ? *m : *n;
    auto Am = SUB(A, na, na);
    auto Bm = SUB(B, *m, *n);
    auto Cm = SUB(C, *m, *n);
    if (herm) hemm(side_of(side), *alpha, HermitianMatrix<T>(uplo_of(uplo), Am), Bm, *beta, Cm, sl_opts());
    else symm(side_of(side), *alpha, SymmetricMatrix<T>(uplo_of(uplo), Am), Bm, *beta, Cm, sl_opts());
    done(Cm);
}

template <typename T>
void pherk(bool herm, char const* uplo, char const* trans, int const* n, int const* k, T const* alpha, T* A,
           int const* iA, int const* jA, int const* descA, T const* beta, T* C, int const* iC, int const* jC,
           int const* descC) {
    Op o = op_of(trans);
    auto Am = SUB(A, o == Op::NoTrans ? *n : *k, o == Op::NoTrans ? *k : *n);
    Matrix<T> Ao = o == Op::NoTrans ? Am : (herm ? conj_transpose(Am) : transpose(Am));
    auto Cm = SUB(C, *n, *n);
    if (herm) { HermitianMatrix<T> H(uplo_of(uplo), Cm); herk(std::real(*alpha), Ao, std::real(*beta), H, sl_opts()); }
    else { SymmetricMatrix<T> S(uplo_of(uplo), Cm); syrk(*alpha, Ao, *beta, S, sl_opts()); }
    done(Cm);
}

template <typename T>
void pher2k(bool herm, char const* uplo, char const* trans, int const* n, int const* k, T const* alpha, T* A,
            int const* iA, int const* jA, int const* descA, T* B, int const* iB, int const* jB, int const* descB,
            T const* beta, T* C, int const* iC, int const* jC, int const* descC) {
    Op o = op_of(trans);
    int64_t r = o == Op::NoTrans ? *n : *k, c = o == Op::NoTrans ? *k : *n;
    auto Am = SUB(A, r, c);
    auto Bm = SUB(B, r, c);
    Matrix<T> Ao = o == Op::NoTrans ? Am : (herm ? conj_transpose(Am) : transpose(Am));
    Matrix<T> Bo = o == Op::NoTrans ? Bm : (herm ? conj_transpose(Bm) : transpose(Bm));
    auto Cm = SUB(C, *n, *n);
    if (herm) { HermitianMatrix<T> H(uplo_of(uplo), Cm); her2k(*alpha, Ao, Bo, std::real(*beta), H, sl_opts()); }
    else { SymmetricMatrix<T> S(uplo_of(uplo), Cm); syr2k(*alpha, Ao, Bo, *beta, S, sl_opts()); }
    done(Cm);
}

template <typename T>
void ptrmm(bool solve, char const* side, char const* uplo, char const* transa, char const* diag, int const* m,
           int const* n, T const* alpha, T* A, int const* iA, int const* jA, int const* descA, T* B,
           int const* iB, int const* jB, int const* descB) {
    int64_t na = side_of(side) == Side::Left ? *m : *n;
    auto Am = SUB(A, na, na);
    auto Bm = SUB(B, *m, *n);
    TriangularMatrix<T> Tm(uplo_of(uplo), diag_of(diag), Am);
    Op o = op_of(transa);
    TriangularMatrix<T> To = o == Op::NoTrans ? Tm : o == Op::Trans ? transpose(Tm) : conj_transpose(Tm);
    if (solve) trsm(side_of(side), *alpha, To, Bm, sl_opts());
    else trmm(side_of(side), *alpha, To, Bm, sl_opts());
    done(Bm);
}

template <typename T>
void pgetrf(int const* m, int const* n, T* A, int const* iA, int const* jA, int const* descA, int* ipiv, int* info) {
    auto Am = SUB(A, *m, *n);
    Pivots P;
    *info = int(getrf(Am, P, sl_opts()));
    done(Am);
    to_ipiv(Am, P, ipiv);
}

template <typename T>
void pgetrs(char const* trans, int const* n, int const* nrhs, T* A, int const* iA, int const* jA,
            int const* descA, int const* ipiv, T* B, int const* iB, int const* jB, int const* descB, int* info) {
    auto Am = SUB(A, *n, *n);
    auto Bm = SUB(B, *n, *nrhs);
    Pivots P = from_ipiv(Am, *n, ipiv);
    getrs(op_of(trans), Am, P, Bm, sl_opts());
    done(Bm);
    *info = 0;
}

template <typename T>
void pgesv(int const* n, int const* nrhs, T* A, int const* iA, int const* jA, int const* descA, int* ipiv, T* B,
           int const* iB, int const* jB, int const* descB, int* info) {
    auto Am = SUB(A, *n, *n);
    auto Bm = SUB(B, *n, *nrhs);
    Pivots P;
    *info = int(gesv(Am, P, Bm, sl_opts()));
    done(Am);
    done(Bm);
    to_ipiv(Am, P, ipiv);
}

/// Mixed-precision solve, ScaLAPACK p?gesv_mixed naming of the reference
/// (scalapack_api/scalapack_gesv_mixed.cc): pdsgesv / pzcgesv.  A is factored
/// in the lower precision (A's tiles keep the original fp64 values; the
/// factors live in a separate low-precision copy), X gets the refined solution,
/// iter the refinement count (negative: fell back to the full-precision LU).
template <typename T>
void pgesv_mixed(int const* n, int const* nrhs, T* A, int const* iA, int const* jA, int const* descA, int* ipiv,
                 T* B, int const* iB, int const* jB, int const* descB, T* X, int const* iX, int const* jX,
                 int const* descX, int* iter, int* info) {
    auto Am = SUB(A, *n, *n);
    auto Bm = SUB(B, *n, *nrhs);
    auto Xm = SUB(X, *n, *nrhs);
    Pivots P;
    int it = 0;
    *info = int(gesv_mixed(Am, P, Bm, Xm, it, sl_opts()));
    *iter = it;
    done(Am);
    done(Xm);
    to_ipiv(Am, P, ipiv);
}

template <typename T>
void pgetri(int const* n, T* A, int const* iA, int const* jA, int const* descA, int const* ipiv, int* info) {
    auto Am = SUB(A, *n, *n);
    Pivots P = from_ipiv(Am, *n, ipiv);
    *info = int(getri(Am, P, sl_opts()));
    done(Am);
}

template <typename T>
void ppotrf(char const* uplo, int const* n, T* A, int const* iA, int const* jA, int const* descA, int* info) {
    auto Am = SUB(A, *n, *n);
    HermitianMatrix<T> H(uplo_of(uplo), Am);
    *info = int(potrf(H, sl_opts()));
    done(Am);
}

template <typename T>
void ppotrs(char const* uplo, int const* n, int const* nrhs, T* A, int const* iA, int const* jA, int const* descA,
            T* B, int const* iB, int const* jB, int const* descB, int* info) {
    auto Am = SUB(A, *n, *n);
    auto Bm = SUB(B, *n, *nrhs);
    HermitianMatrix<T> H(uplo_of(uplo), Am);
    potrs(H, Bm, sl_opts());
    done(Bm);
    *info = 0;
}

template <typename T>
void pposv(char const* uplo, int const* n, int const* nrhs, T* A, int const* iA, int const* jA, int const* descA,
           T* B, int const* iB, int const* jB, int const* descB, int* info) {
    auto Am = SUB(A, *n, *n);
    auto Bm = SUB(B, *n, *nrhs);
    HermitianMatrix<T> H(uplo_of(uplo), Am);
    *info = int(posv(H, Bm, sl_opts()));
    done(Am);
    done(Bm);
}

template <typename T>
void ppotri(char const* uplo, int const* n, T* A, int const* iA, int const* jA, int const* descA, int* info) {
    auto Am = SUB(A, *n, *n);
    HermitianMatrix<T> H(uplo_of(uplo), Am);
    *info = int(potri(H, sl_opts()));
    done(Am);
}

template <typename T>
void pgels(char const* trans, int const* m, int const* n, int const* nrhs, T* A, int const* iA, int const* jA,
           int const* descA, T* B, int const* iB, int const* jB, int const* descB, int* info) {
    *info = 0;
    if (op_of(trans) != Op::NoTrans) { *info = -1; return; }
    auto Am = SUB(A, *m, *n);
    auto Bm = SUB(B, std::max(*m, *n), *nrhs);
    TriangularFactors<T> Tf;
    gels(Am, Tf, Bm, sl_opts());
    done(Am);
    done(Bm);
}

template <typename T>
real_type<T> plange(char const* norm, int const* m, int const* n, T* A, int const* iA, int const* jA,
                    int const* descA) {
    auto Am = SUB(A, *m, *n);
    return slate::norm(norm_of(norm), Am, sl_opts());
}

template <typename T>
real_type<T> planhe(bool herm, char const* norm, char const* uplo, int const* n, T* A, int const* iA,
                    int const* jA, int const* descA) {
    auto Am = SUB(A, *n, *n);
    if (herm) return slate::norm(norm_of(norm), HermitianMatrix<T>(uplo_of(uplo), Am), sl_opts());
    return slate::norm(norm_of(norm), SymmetricMatrix<T>(uplo_of(uplo), Am), sl_opts());
}

template <typename T>
real_type<T> plantr(char const* norm, char const* uplo, char const* diag, int const* m, int const* n, T* A,
                    int const* iA, int const* jA, int const* descA) {
    auto Am = SUB(A, *m, *n);
    return slate::norm(norm_of(norm), TrapezoidMatrix<T>(uplo_of(uplo), diag_of(diag), Am), sl_opts());
}

template <typename T>
void pgecon(char const* norm, int const* n, T* A, int const* iA, int const* jA, int const* descA,
            real_type<T> const* anorm, real_type<T>* rcond, int* info) {
    auto Am = SUB(A, *n, *n);
    *rcond = gecondest(norm_of(norm), Am, *anorm, sl_opts());
    *info = 0;
}

template <typename T>
void ppocon(char const* uplo, int const* n, T* A, int const* iA, int const* jA, int const* descA,
            real_type<T> const* anorm, real_type<T>* rcond, int* info) {
    auto Am = SUB(A, *n, *n);
    HermitianMatrix<T> H(uplo_of(uplo), Am);
    *rcond = pocondest(Norm::One, H, *anorm, sl_opts());
    *info = 0;
}

template <typename T>
void ptrcon(char const* norm, char const* uplo, char const* diag, int const* n, T* A, int const* iA,
            int const* jA, int const* descA, real_type<T>* rcond, int* info) {
    auto Am = SUB(A, *n, *n);
    TriangularMatrix<T> Tm(uplo_of(uplo), diag_of(diag), Am);
    *rcond = trcondest(norm_of(norm), Tm, sl_opts());
    *info = 0;
}

template <typename T>
void pheev(char const* jobz, char const* uplo, int const* n, T* A, int const* iA, int const* jA, int const* descA,
           real_type<T>* W, T* Z, int const* iZ, int const* jZ, int const* descZ, int* info) {
    auto Am = SUB(A, *n, *n);
    HermitianMatrix<T> H(uplo_of(uplo), Am);
    std::vector<real_type<T>> L;
    Matrix<T> Zm;
    if (up(jobz) == 'V') Zm = SUB(Z, *n, *n);
    heev(H, L, Zm, sl_opts());
    std::copy(L.begin(), L.end(), W);
    if (up(jobz) == 'V') done(Zm);
    *info = 0;
}

template <typename T>
void pgesvd(char const* jobu, char const* jobvt, int const* m, int const* n, T* A, int const* iA, int const* jA,
            int const* descA, real_type<T>* S, T* U, int const* iU, int const* jU, int const* descU, T* VT,
            int const* iVT, int const* jVT, int const* descVT, int* info) {
    *info = 0;
    const int64_t k = std::min(*m, *n);
    auto Am = SUB(A, *m, *n);
    Matrix<T> Um, Vm;
    if (up(jobu) == 'V') Um = SUB(U, *m, k);
    if (up(jobvt) == 'V') Vm = SUB(VT, k, *n);
    std::vector<real_type<T>> Sv;
    svd(Am, Sv, Um, Vm, sl_opts());
    std::copy(Sv.begin(), Sv.end(), S);
    if (up(jobu) == 'V') done(Um);
    if (up(jobvt) == 'V') done(Vm);
}

#undef SUB

// Hermitian rank-k/2k take real alpha/beta in ScaLAPACK
template <typename T>
void pherk_r(char const* ul, char const* tr, int const* n, int const* k, real_type<T> const* al, T* A,
             int const* iA, int const* jA, int const* descA, real_type<T> const* be, T* C, int const* iC,
             int const* jC, int const* descC) {
    T a(*al), b(*be);
    pherk<T>(true, ul, tr, n, k, &a, A, iA, jA, descA, &b, C, iC, jC, descC);
}
template <typename T>
void pher2k_r(char const* ul, char const* tr, int const* n, int const* k, T const* al, T* A, int const* iA,
              int const* jA, int const* descA, T* B, int const* iB, int const* jB, int const* descB,
              real_type<T> const* be, T* C, int const* iC, int const* jC, int const* descC) {
    T b(*be);
    pher2k<T>(true, ul, tr, n, k, al, A, iA, jA, descA, B, iB, jB, descB, &b, C, iC, jC, descC);
}

}  // namespace

// Every routine is exported as p<x>name_, p<x>name and P<X>NAME (Fortran
// compilers differ), all forwarding to the templates above.
#define SL3(ret, lname, uname, params, call)                                                                \
    extern "C" ret lname##_ params { return call; }                                                          \
    extern "C" ret lname params { return call; }                                                             \
    extern "C" ret uname params { return call; }

#define DESC(X) T* X, int const* i##X, int const* j##X, int const* desc##X
#define DARGS(X) X, i##X, j##X, desc##X

#define SLATE_SCALAPACK_API(p, P, T)                                                                         \
SL3(void, p##gemm, P##GEMM, (char const* ta, char const* tb, int const* m, int const* n, int const* k,      \
    T const* al, DESC(A), DESC(B), T const* be, DESC(C)),                                                    \
    pgemm<T>(ta, tb, m, n, k, al, DARGS(A), DARGS(B), be, DARGS(C)))                                         \
SL3(void, p##symm, P##SYMM, (char const* sd, char const* ul, int const* m, int const* n, T const* al,       \
    DESC(A), DESC(B), T const* be, DESC(C)),                                                                 \
    phemm<T>(false, sd, ul, m, n, al, DARGS(A), DARGS(B), be, DARGS(C)))                                     \
SL3(void, p##syrk, P##SYRK, (char const* ul, char const* tr, int const* n, int const* k, T const* al,       \
    DESC(A), T const* be, DESC(C)), pherk<T>(false, ul, tr, n, k, al, DARGS(A), be, DARGS(C)))              \
SL3(void, p##syr2k, P##SYR2K, (char const* ul, char const* tr, int const* n, int const* k, T const* al,     \
    DESC(A), DESC(B), T const* be, DESC(C)),                                                                 \
    pher2k<T>(false, ul, tr, n, k, al, DARGS(A), DARGS(B), be, DARGS(C)))                                    \
SL3(void, p##trmm, P##TRMM, (char const* sd, char const* ul, char const* ta, char const* dg, int const* m,  \
    int const* n, T const* al, DESC(A), DESC(B)),                                                            \
    ptrmm<T>(false, sd, ul, ta, dg, m, n, al, DARGS(A), DARGS(B)))                                           \
SL3(void, p##trsm, P##TRSM, (char const* sd, char const* ul, char const* ta, char const* dg, int const* m,  \
    int const* n, T const* al, DESC(A), DESC(B)),                                                            \
    ptrmm<T>(true, sd, ul, ta, dg, m, n, al, DARGS(A), DARGS(B)))                                            \
SL3(void, p##getrf, P##GETRF, (int const* m, int const* n, DESC(A), int* ipiv, int* info),                  \
    pgetrf<T>(m, n, DARGS(A), ipiv, info))                                                                   \
SL3(void, p##getrs, P##GETRS, (char const* tr, int const* n, int const* nrhs, DESC(A), int const* ipiv,     \
    DESC(B), int* info), pgetrs<T>(tr, n, nrhs, DARGS(A), ipiv, DARGS(B), info))                             \
SL3(void, p##gesv, P##GESV, (int const* n, int const* nrhs, DESC(A), int* ipiv, DESC(B), int* info),        \
    pgesv<T>(n, nrhs, DARGS(A), ipiv, DARGS(B), info))                                                       \
SL3(void, p##getri, P##GETRI, (int const* n, DESC(A), int const* ipiv, T*, int const*, int*, int const*,    \
    int* info), pgetri<T>(n, DARGS(A), ipiv, info))                                                          \
SL3(void, p##potrf, P##POTRF, (char const* ul, int const* n, DESC(A), int* info),                           \
    ppotrf<T>(ul, n, DARGS(A), info))                                                                        \
SL3(void, p##potrs, P##POTRS, (char const* ul, int const* n, int const* nrhs, DESC(A), DESC(B), int* info), \
    ppotrs<T>(ul, n, nrhs, DARGS(A), DARGS(B), info))                                                        \
SL3(void, p##posv, P##POSV, (char const* ul, int const* n, int const* nrhs, DESC(A), DESC(B), int* info),   \
    pposv<T>(ul, n, nrhs, DARGS(A), DARGS(B), info))                                                         \
SL3(void, p##potri, P##POTRI, (char const* ul, int const* n, DESC(A), int* info),                           \
    ppotri<T>(ul, n, DARGS(A), info))                                                                        \
SL3(void, p##gels, P##GELS, (char const* tr, int const* m, int const* n, int const* nrhs, DESC(A), DESC(B), \
    T*, int const*, int* info), pgels<T>(tr, m, n, nrhs, DARGS(A), DARGS(B), info))                         \
SL3(real_type<T>, p##lange, P##LANGE, (char const* nm, int const* m, int const* n, DESC(A), real_type<T>*), \
    plange<T>(nm, m, n, DARGS(A)))                                                                           \
SL3(real_type<T>, p##lansy, P##LANSY, (char const* nm, char const* ul, int const* n, DESC(A),               \
    real_type<T>*), planhe<T>(false, nm, ul, n, DARGS(A)))                                                   \
SL3(real_type<T>, p##lantr, P##LANTR, (char const* nm, char const* ul, char const* dg, int const* m,         \
    int const* n, DESC(A), real_type<T>*), plantr<T>(nm, ul, dg, m, n, DARGS(A)))                           \
SL3(void, p##gecon, P##GECON, (char const* nm, int const* n, DESC(A), real_type<T> const* an,              \
    real_type<T>* rc, T*, int const*, void*, int const*, int* info),                                        \
    pgecon<T>(nm, n, DARGS(A), an, rc, info))                                                                \
SL3(void, p##pocon, P##POCON, (char const* ul, int const* n, DESC(A), real_type<T> const* an,              \
    real_type<T>* rc, T*, int const*, void*, int const*, int* info),                                        \
    ppocon<T>(ul, n, DARGS(A), an, rc, info))                                                                \
SL3(void, p##trcon, P##TRCON, (char const* nm, char const* ul, char const* dg, int const* n, DESC(A),       \
    real_type<T>* rc, T*, int const*, void*, int const*, int* info),                                        \
    ptrcon<T>(nm, ul, dg, n, DARGS(A), rc, info))                                                            \
SL3(void, p##gesvd, P##GESVD, (char const* ju, char const* jv, int const* m, int const* n, DESC(A),         \
    real_type<T>* S, DESC(U), DESC(VT), T*, int const*, int* info),                                         \
    pgesvd<T>(ju, jv, m, n, DARGS(A), S, DARGS(U), DARGS(VT), info))

// p?gesv_mixed: only the fp64 -> fp32 pairs exist (pdsgesv, pzcgesv)
#define SLATE_SCALAPACK_API_MIXED(name, NAME, T)                                                             \
SL3(void, name, NAME, (int const* n, int const* nrhs, DESC(A), int* ipiv, DESC(B), DESC(X), int* iter,       \
    int* info), pgesv_mixed<T>(n, nrhs, DARGS(A), ipiv, DARGS(B), DARGS(X), iter, info))

#define SLATE_SCALAPACK_API_REAL(p, P, T)                                                                    \
SL3(void, p##syev, P##SYEV, (char const* jz, char const* ul, int const* n, DESC(A), T* W, DESC(Z), T*,      \
    int const*, int* info), pheev<T>(jz, ul, n, DARGS(A), W, DARGS(Z), info))                               \
SL3(void, p##syevd, P##SYEVD, (char const* jz, char const* ul, int const* n, DESC(A), T* W, DESC(Z), T*,    \
    int const*, int*, int const*, int* info), pheev<T>(jz, ul, n, DARGS(A), W, DARGS(Z), info))

#define SLATE_SCALAPACK_API_CPLX(p, P, T)                                                                    \
SL3(void, p##hemm, P##HEMM, (char const* sd, char const* ul, int const* m, int const* n, T const* al,       \
    DESC(A), DESC(B), T const* be, DESC(C)),                                                                 \
    phemm<T>(true, sd, ul, m, n, al, DARGS(A), DARGS(B), be, DARGS(C)))                                      \
SL3(void, p##herk, P##HERK, (char const* ul, char const* tr, int const* n, int const* k,                     \
    real_type<T> const* al, DESC(A), real_type<T> const* be, DESC(C)),                                      \
    pherk_r<T>(ul, tr, n, k, al, DARGS(A), be, DARGS(C)))                   \
SL3(void, p##her2k, P##HER2K, (char const* ul, char const* tr, int const* n, int const* k, T const* al,      \
    DESC(A), DESC(B), real_type<T> const* be, DESC(C)),                                                      \
    pher2k_r<T>(ul, tr, n, k, al, DARGS(A), DARGS(B), be, DARGS(C)))                \
SL3(real_type<T>, p##lanhe, P##LANHE, (char const* nm, char const* ul, int const* n, DESC(A),               \
    real_type<T>*), planhe<T>(true, nm, ul, n, DARGS(A)))                                                    \
SL3(void, p##heev, P##HEEV, (char const* jz, char const* ul, int const* n, DESC(A), real_type<T>* W,        \
    DESC(Z), T*, int const*, real_type<T>*, int const*, int* info),                                         \
    pheev<T>(jz, ul, n, DARGS(A), W, DARGS(Z), info))                                                        \
SL3(void, p##heevd, P##HEEVD, (char const* jz, char const* ul, int const* n, DESC(A), real_type<T>* W,      \
    DESC(Z), T*, int const*, real_type<T>*, int const*, int*, int const*, int* info),                       \
    pheev<T>(jz, ul, n, DARGS(A), W, DARGS(Z), info))

namespace {
using s_t = float;
using d_t = double;
using c_t = std::complex<float>;
using z_t = std::complex<double>;
}

#define T s_t
SLATE_SCALAPACK_API(ps, PS, T)
SLATE_SCALAPACK_API_REAL(ps, PS, T)
#undef T
#define T d_t
SLATE_SCALAPACK_API(pd, PD, T)
SLATE_SCALAPACK_API_REAL(pd, PD, T)
SLATE_SCALAPACK_API_MIXED(pdsgesv, PDSGESV, T)
#undef T
#define T c_t
SLATE_SCALAPACK_API(pc, PC, T)
SLATE_SCALAPACK_API_CPLX(pc, PC, T)
#undef T
#define T z_t
SLATE_SCALAPACK_API(pz, PZ, T)
SLATE_SCALAPACK_API_CPLX(pz, PZ, T)
SLATE_SCALAPACK_API_MIXED(pzcgesv, PZCGESV, T)
#undef T
