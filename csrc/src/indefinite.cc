// Hermitian indefinite factorization and solve (reference src/hetrf.cc,
// hetrs.cc, hesv.cc).
//
// hetrf(A, pivots, T, pivots2, H): blocked left-looking Aasen, distributed
// and device-resident (reference hetrf.cc):  P A P^T = L T L^H with L unit
// lower (first block column [I; 0]) and T Hermitian block tridiagonal.  A is
// only ever read one (symmetrically permuted) block column per step, so the
// permutation is never applied to the trailing matrix: step k gathers
// F(perm[kk:], perm[kk:kk+nb]) (O(n nb) data), forms H(:, k) = T L(k, :)^H
// from the replicated T and block row of L, computes T(k, k), updates the
// panel W = A(k+1:, k) - L(k+1:, :) H(:, k) with a distributed GEMM
// (row-reduced), factors it with the distributed partial-pivoting LU
// (getrf on the panel), and applies the pivots to L's left block columns.
// T is band-LU factored (gbtrf, pivots2); hetrs applies P, L, T, L^H, P^T.
//
// hetrf(A, ipiv): Bunch-Kaufman diagonal pivoting, A = P L D L^H P^T with
// 1x1 and 2x2 pivots (LAPACK hetf2 semantics, host, replicated), LAPACK ipiv.
#include "internal.hh"
#include "../kernels/kernels.hh"

#include <cmath>

namespace slate {

using namespace internal;

namespace {

template <typename T> inline real_type<T> cabs1(T x) { return std::abs(std::real(x)) + std::abs(std::imag(x)); }

/// Lower Bunch-Kaufman on a dense column-major n x n array.
template <typename T>
int64_t hetf2_lower(int64_t n, T* a, int64_t lda, int64_t* ipiv) {
    using R = real_type<T>;
    auto A = [&](int64_t i, int64_t j) -> T& { return a[i + j * lda]; };
    const R alpha = (R(1) + std::sqrt(R(17))) / R(8);
    int64_t info = 0, k = 0;
    while (k < n) {
        int64_t kstep = 1, kp = k;
        R absakk = std::abs(std::real(A(k, k)));
        int64_t imax = k;
        R colmax = 0;
        for (int64_t i = k + 1; i < n; ++i) if (cabs1(A(i, k)) > colmax) { colmax = cabs1(A(i, k)); imax = i; }
        if (std::max(absakk, colmax) == R(0)) {
            if (info == 0) info = k + 1;
            kp = k;
            A(k, k) = T(std::real(A(k, k)));
        } else {
            if (absakk >= alpha * colmax) {
                kp = k;
            } else {
                R rowmax = 0;
                for (int64_t j = k; j < imax; ++j) rowmax = std::max(rowmax, cabs1(A(imax, j)));
                for (int64_t i = imax + 1; i < n; ++i) rowmax = std::max(rowmax, cabs1(A(i, imax)));
                if (absakk >= alpha * colmax * (colmax / rowmax)) kp = k;
                else if (std::abs(std::real(A(imax, imax))) >= alpha * rowmax) kp = imax;
                else { kp = imax; kstep = 2; }
            }
            const int64_t kk = k + kstep - 1;
            if (kp != kk) {
                for (int64_t i = kp + 1; i < n; ++i) std::swap(A(i, kk), A(i, kp));
                for (int64_t j = kk + 1; j < kp; ++j) {
                    T t = slate::conj(A(j, kk));
                    A(j, kk) = slate::conj(A(kp, j));
                    A(kp, j) = t;
                }
                A(kp, kk) = slate::conj(A(kp, kk));
                R r1 = std::real(A(kk, kk));
                A(kk, kk) = T(std::real(A(kp, kp)));
                A(kp, kp) = T(r1);
                if (kstep == 2) {
                    A(k, k) = T(std::real(A(k, k)));
                    std::swap(A(k + 1, k), A(kp, k));
                }
            } else {
                A(k, k) = T(std::real(A(k, k)));
                if (kstep == 2) A(k + 1, k + 1) = T(std::real(A(k + 1, k + 1)));
            }
            if (kstep == 1) {
                R r1 = R(1) / std::real(A(k, k));
                #pragma omp parallel for schedule(static) if (n - k > 256)
                for (int64_t j = k + 1; j < n; ++j) {
                    T xj = slate::conj(A(j, k)) * r1;
                    for (int64_t i = j; i < n; ++i) A(i, j) -= A(i, k) * xj;
                    A(j, j) = T(std::real(A(j, j)));
                }
                for (int64_t i = k + 1; i < n; ++i) A(i, k) *= r1;
            } else if (k + 2 < n) {
                R d = std::abs(A(k + 1, k));
                R d11 = std::real(A(k + 1, k + 1)) / d;
                R d22 = std::real(A(k, k)) / d;
                R tt = R(1) / (d11 * d22 - R(1));
                T d21 = A(k + 1, k) / d;
                R dd = tt / d;
                std::vector<T> wk(n), wkp1(n);
                for (int64_t j = k + 2; j < n; ++j) {
                    wk[j] = dd * (d11 * A(j, k) - d21 * A(j, k + 1));
                    wkp1[j] = dd * (d22 * A(j, k + 1) - slate::conj(d21) * A(j, k));
                }
                #pragma omp parallel for schedule(static) if (n - k > 256)
                for (int64_t j = k + 2; j < n; ++j) {
                    T cw = slate::conj(wk[j]), cw1 = slate::conj(wkp1[j]);
                    for (int64_t i = j; i < n; ++i) A(i, j) -= A(i, k) * cw + A(i, k + 1) * cw1;
                    A(j, j) = T(std::real(A(j, j)));
                }
                for (int64_t j = k + 2; j < n; ++j) { A(j, k) = wk[j]; A(j, k + 1) = wkp1[j]; }
            }
        }
        if (kstep == 1) ipiv[k] = kp + 1;
        else ipiv[k] = ipiv[k + 1] = -(kp + 1);
        k += kstep;
    }
    return info;
}

template <typename T>
void hetrs_lower(int64_t n, int64_t nrhs, T const* a, int64_t lda, int64_t const* ipiv, T* b, int64_t ldb) {
    auto A = [&](int64_t i, int64_t j) { return a[i + j * lda]; };
    #pragma omp parallel for schedule(static) if (nrhs > 1)
    for (int64_t c = 0; c < nrhs; ++c) {
        T* x = b + c * ldb;
        int64_t k = 0;
        while (k < n) {
            if (ipiv[k] > 0) {
                int64_t kp = ipiv[k] - 1;
                if (kp != k) std::swap(x[k], x[kp]);
                for (int64_t i = k + 1; i < n; ++i) x[i] -= A(i, k) * x[k];
                x[k] /= std::real(A(k, k));
                k += 1;
            } else {
                int64_t kp = -ipiv[k] - 1;
                if (kp != k + 1) std::swap(x[k + 1], x[kp]);
                for (int64_t i = k + 2; i < n; ++i) x[i] -= A(i, k) * x[k] + A(i, k + 1) * x[k + 1];
                T akm1k = A(k + 1, k);
                T akm1 = A(k, k) / slate::conj(akm1k);
                T ak = A(k + 1, k + 1) / akm1k;
                T denom = akm1 * ak - T(1);
                T bkm1 = x[k] / slate::conj(akm1k);
                T bk = x[k + 1] / akm1k;
                x[k] = (ak * bkm1 - bk) / denom;
                x[k + 1] = (akm1 * bk - bkm1) / denom;
                k += 2;
            }
        }
        k = n - 1;
        while (k >= 0) {
            if (ipiv[k] > 0) {
                T s = x[k];
                for (int64_t i = k + 1; i < n; ++i) s -= slate::conj(A(i, k)) * x[i];
                x[k] = s;
                int64_t kp = ipiv[k] - 1;
                if (kp != k) std::swap(x[k], x[kp]);
                k -= 1;
            } else {
                T s = x[k], s1 = x[k - 1];
                for (int64_t i = k + 1; i < n; ++i) {
                    s -= slate::conj(A(i, k)) * x[i];
                    s1 -= slate::conj(A(i, k - 1)) * x[i];
                }
                x[k] = s;
                x[k - 1] = s1;
                int64_t kp = -ipiv[k] - 1;
                if (kp != k) std::swap(x[k], x[kp]);
                k -= 2;
            }
        }
    }
}

/// Replicated lower-triangle copy of a Hermitian matrix (Upper read as L^H).
template <typename T>
std::vector<T> gather_lower(HermitianMatrix<T> const& A, Options const& opts) {
    Matrix<T> G(A);
    G.set_uplo(Uplo::General);
    std::vector<T> full;
    gather(G, full, opts);
    const int64_t n = A.n();
    if (A.uplo() == Uplo::Upper)
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = j; i < n; ++i) full[i + j * n] = slate::conj(full[j + i * n]);
    return full;
}

}  // namespace

template <typename T>
int64_t hetrf(HermitianMatrix<T>& A, std::vector<int64_t>& ipiv, Options const& opts) {
    trace::Block tb("hetrf");
    internal::DriverScope ds_;
    const int64_t n = A.n();
    std::vector<T> a = gather_lower(A, opts);
    ipiv.assign(n, 0);
    int64_t info = hetf2_lower<T>(n, a.data(), n, ipiv.data());
    // write back the factor into A's stored triangle
    Matrix<T> G(A);
    G.set_uplo(Uplo::General);
    const bool upper = A.uplo() == Uplo::Upper;
    Options oh = {{Option::Target, Target::Host}};
    set<T>(std::function<T(int64_t, int64_t)>([&](int64_t i, int64_t j) {
        if (!upper) return i >= j ? a[i + j * n] : T(0);
        return i <= j ? slate::conj(a[j + i * n]) : T(0);
    }), G, oh);
    if (resolve_target(opts) == Target::Devices) G.storage()->get(Loc::Device, false);
    return info;
}

template <typename T>
void hetrs(HermitianMatrix<T> const& A, std::vector<int64_t> const& ipiv, Matrix<T>& B, Options const& opts) {
    trace::Block tb("hetrs");
    internal::DriverScope ds_;
    const int64_t n = A.n(), nrhs = B.n();
    std::vector<T> a = gather_lower(A, opts);
    std::vector<T> b;
    gather(B, b, opts);
    hetrs_lower<T>(n, nrhs, a.data(), n, ipiv.data(), b.data(), n);
    Options oh = {{Option::Target, Target::Host}};
    set<T>(std::function<T(int64_t, int64_t)>([&](int64_t i, int64_t j) { return b[i + j * n]; }), B, oh);
    if (resolve_target(opts) == Target::Devices) B.storage()->get(Loc::Device, false);
}

template <typename T>
int64_t hesv(HermitianMatrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B, Options const& opts) {
    trace::Block tb("hesv");
    internal::DriverScope ds_;
    int64_t info = hetrf(A, ipiv, opts);
    if (info == 0) hetrs(A, ipiv, B, opts);
    return info;
}

//------------------------------------------------------------------------------
namespace {

namespace kd = slate_amd::dev;

/// indexed gather dst[rd[a] + cd[b] ldd] = src[ri[a] + ci[b] lds] (host or device)
template <typename T>
void gather_idx(lb::Ctx const& c, std::vector<int64_t> const& ri, std::vector<int64_t> const& ci, T const* src,
                int64_t lds, std::vector<int64_t> const& rd, std::vector<int64_t> const& cd, T* dst, int64_t ldd) {
    if (ri.empty() || ci.empty()) return;
    if (!c.dev()) {
        for (size_t b = 0; b < ci.size(); ++b)
            for (size_t a = 0; a < ri.size(); ++a) dst[rd[a] + cd[b] * ldd] = src[ri[a] + ci[b] * lds];
        return;
    }
    std::vector<int64_t> h;
    h.reserve(2 * (ri.size() + ci.size()));
    h.insert(h.end(), ri.begin(), ri.end());
    h.insert(h.end(), ci.begin(), ci.end());
    h.insert(h.end(), rd.begin(), rd.end());
    h.insert(h.end(), cd.begin(), cd.end());
    Work<int64_t> d(Target::Devices, h.size());
    device::memcpy_async(d.data(), h.data(), h.size() * sizeof(int64_t), c.stream);
    const size_t nr = ri.size(), nc = ci.size();
    kd::gather2d(int64_t(nr), int64_t(nc), kd::dptr(src), lds, d.data(), d.data() + nr, kd::dptr(dst), ldd,
                 d.data() + nr + nc, d.data() + 2 * nr + nc, c.stream);
    slate_hip_call(hipStreamSynchronize(c.stream));
}

template <typename T>
inline void sum_world(Comm& w, T* buf, size_t n, lb::Ctx const& c) {
    if (w.size() > 1 && n > 0) w.allreduce(buf, buf, n, scalar_type<T>(), ReduceOp::Sum, c.loc(), c.stream);
}

}  // namespace

template <typename T>
int64_t hetrf(HermitianMatrix<T>& A, Pivots& pivots, BandMatrix<T>& Tb, Pivots& pivots2, Matrix<T>& H,
              Options const& opts) {
    trace::Block tb("hetrf_aasen");
    internal::DriverScope ds_;
    (void)H;
    Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    slate_error_if_msg(A.uplo() != Uplo::Lower, "hetrf (Aasen): Lower storage required (as the reference)");
    slate_error_if_msg(A.op() != Op::NoTrans || !A.aligned() || A.mb() != A.nb(),
                       "hetrf (Aasen): NoTrans, tile-aligned, square-tile matrix required");
    const int64_t n = A.n(), nb = A.nb(), nt = A.nt();
    auto gp = A.grid();
    auto& g = *gp;
    Comm& world = g.world();
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    // full Hermitian copy F (read only): the permuted block columns come from it
    Matrix<T> Ag(A);
    Ag.set_uplo(Uplo::General);
    Matrix<T> F = Ag.emptyLike();
    F.insertLocalTiles(target);
    slate::copy<T, T>(conj_transpose(Ag), F, opts);
    {
        BaseTrapezoidMatrix<T> At(Uplo::Lower, Ag, MatrixKind::Trapezoid), Ft(Uplo::Lower, F, MatrixKind::Trapezoid);
        slate::copy<T, T>(At, Ft, opts);
    }
    // L overwrites A's storage: zero, L(0, 0) = I
    Matrix<T> Lm = Ag;
    set(T(0), T(0), Lm, opts);
    {
        Matrix<T> L00 = Lm.sub(0, 0, 0, 0);
        set(T(0), T(1), L00, opts);
    }
    LocalBlock<T> lf = F.local(loc, false);
    auto& st = *Lm.storage();
    const int64_t mloc = lf.m, nloc = lf.n;
    std::vector<int64_t> rowg(mloc), colg(nloc);
    for (int64_t li = 0; li < mloc; ++li) rowg[li] = l2g(li, st.mb, st.rrel(), g.p());
    for (int64_t lj = 0; lj < nloc; ++lj) colg[lj] = l2g(lj, st.nb, st.crel(), g.q());
    // replicated T blocks: Td[k] = T(k, k), Ts[k] = T(k+1, k) (nb x nb each)
    Work<T> Td(target, size_t(nb * nb) * nt), Ts(target, size_t(nb * nb) * nt);
    lb::set(c, Uplo::General, nb * nb, nt, T(0), T(0), Td.data(), nb * nb);
    lb::set(c, Uplo::General, nb * nb, nt, T(0), T(0), Ts.data(), nb * nb);
    auto tdiag = [&](int64_t k) { return Td.data() + k * nb * nb; };
    auto tsub = [&](int64_t k) { return Ts.data() + k * nb * nb; };
    Work<T> G(target, size_t(n) * nb), LK(target, size_t(nb) * std::max<int64_t>(n, 1)),
        Hb(target, size_t(n) * nb), Cw(target, size_t(nb) * nb), Xw(target, size_t(nb) * nb),
        Hl(target, size_t(std::max<int64_t>(nloc, 1)) * nb), Pw(target, size_t(std::max<int64_t>(mloc, 1)) * nb),
        Uw(target, size_t(nb) * nb);
    std::vector<int64_t> perm(n), pinv(n);
    for (int64_t i = 0; i < n; ++i) perm[i] = pinv[i] = i;
    pivots.assign(nt, {});
    for (int64_t t = 0; t < A.tileNb(0); ++t) pivots[0].push_back(Pivot(0, t));
    int64_t info = 0;
    for (int64_t k = 0; k < nt; ++k) {
        const int64_t kk = k * nb, wk = A.tileNb(k), ke = kk + wk, mk = n - kk;
        // 1. G = F(perm[kk:], perm[kk:ke]) replicated ((n - kk) x wk, ld mk)
        {
            trace::Block t2("aasen_gather_column");
            std::vector<int64_t> ri, rd, ci, cd;
            for (int64_t li = 0; li < mloc; ++li)
                if (pinv[rowg[li]] >= kk) { ri.push_back(li); rd.push_back(pinv[rowg[li]] - kk); }
            for (int64_t lj = 0; lj < nloc; ++lj) {
                const int64_t p = pinv[colg[lj]];
                if (p >= kk && p < ke) { ci.push_back(lj); cd.push_back(p - kk); }
            }
            lb::set(c, Uplo::General, mk, wk, T(0), T(0), G.data(), mk);
            gather_idx(c, ri, ci, lf.ptr, lf.ld, rd, cd, G.data(), mk);
            sum_world(world, G.data(), size_t(mk) * wk, c);
        }
        // 2. LK = L(kk:ke, 0:ke) replicated (wk x ke, ld nb)
        LocalBlock<T> ll = Lm.local(loc, true);
        {
            std::vector<int64_t> ri, rd, ci, cd;
            for (int64_t li = 0; li < mloc; ++li)
                if (rowg[li] >= kk && rowg[li] < ke) { ri.push_back(li); rd.push_back(rowg[li] - kk); }
            for (int64_t lj = 0; lj < nloc; ++lj)
                if (colg[lj] < ke) { ci.push_back(lj); cd.push_back(colg[lj]); }
            lb::set(c, Uplo::General, nb, ke, T(0), T(0), LK.data(), nb);
            gather_idx(c, ri, ci, ll.ptr, ll.ld, rd, cd, LK.data(), nb);
            sum_world(world, LK.data(), size_t(nb) * ke, c);
        }
        T* Lkk = LK.data() + kk * nb;
        // 3. H(i, k) = T(i, i-1) L(k, i-1)^H + T(i, i) L(k, i)^H + T(i, i+1) L(k, i+1)^H, i < k  (ld n)
        for (int64_t i = 0; i < k; ++i) {
            const int64_t ri0 = i * nb, wi = A.tileNb(i);
            T* Hi = Hb.data() + ri0;
            lb::gemm(c, Op::NoTrans, Op::ConjTrans, wi, wk, wi, T(1), tdiag(i), nb, LK.data() + ri0 * nb, nb, T(0),
                     Hi, n);
            if (i > 0)
                lb::gemm(c, Op::NoTrans, Op::ConjTrans, wi, wk, A.tileNb(i - 1), T(1), tsub(i - 1), nb,
                         LK.data() + (ri0 - nb) * nb, nb, T(1), Hi, n);
            lb::gemm(c, Op::ConjTrans, Op::ConjTrans, wi, wk, A.tileNb(i + 1), T(1), tsub(i), nb,
                     LK.data() + (ri0 + nb) * nb, nb, T(1), Hi, n);
        }
        // 4. T(k, k) = L(k,k)^{-1} [A(k,k) - L(k, 0:k) H(0:k, k) - L(k,k) T(k,k-1) L(k,k-1)^H] L(k,k)^{-H}
        lb::copy2d(c, wk, wk, G.data(), mk, Cw.data(), nb);
        if (k > 0) {
            lb::gemm(c, Op::NoTrans, Op::NoTrans, wk, wk, kk, T(-1), LK.data(), nb, Hb.data(), n, T(1), Cw.data(), nb);
            // Xw = T(k,k-1) L(k,k-1)^H ; C -= L(k,k) Xw
            lb::gemm(c, Op::NoTrans, Op::ConjTrans, wk, wk, A.tileNb(k - 1), T(1), tsub(k - 1), nb,
                     LK.data() + (kk - nb) * nb, nb, T(0), Xw.data(), nb);
            lb::gemm(c, Op::NoTrans, Op::NoTrans, wk, wk, wk, T(-1), Lkk, nb, Xw.data(), nb, T(1), Cw.data(), nb);
        }
        lb::trsm(c, Side::Left, Uplo::Lower, Op::NoTrans, Diag::Unit, wk, wk, T(1), Lkk, nb, Cw.data(), nb);
        lb::trsm(c, Side::Right, Uplo::Lower, Op::ConjTrans, Diag::Unit, wk, wk, T(1), Lkk, nb, Cw.data(), nb);
        lb::copy(c, Uplo::General, Op::ConjTrans, wk, wk, Cw.data(), nb, tdiag(k), nb);
        lb::add(c, Uplo::General, wk, wk, T(0.5), Cw.data(), nb, T(0.5), tdiag(k), nb);    // Hermitian part
        if (ke >= n) break;
        const int64_t w1 = A.tileNb(k + 1), m1 = n - ke;
        // 5. H(k, k) = T(k,k) L(k,k)^H + T(k,k-1) L(k,k-1)^H
        T* Hk = Hb.data() + kk;
        lb::gemm(c, Op::NoTrans, Op::ConjTrans, wk, wk, wk, T(1), tdiag(k), nb, Lkk, nb, T(0), Hk, n);
        if (k > 0) lb::add(c, Uplo::General, wk, wk, T(1), Xw.data(), nb, T(1), Hk, n);
        // 6. W = A(k+1:, k) - L(k+1:, 0:k) H(0:k, k): local GEMM over my columns < ke, row-reduced
        Matrix<T> Wm(m1, wk, nb, wk, gp, Lm.srow_owner(k + 1), Lm.scol_owner(k + 1));
        Wm.insertLocalTiles(target);
        {
            trace::Block t2("aasen_panel_update");
            const int64_t nlc = lcol_of(Lm, k + 1);     // my columns with global index < ke
            std::vector<int64_t> hr, hrd, hc, hcd;
            for (int64_t lj = 0; lj < nlc; ++lj) { hr.push_back(colg[lj]); hrd.push_back(lj); }
            for (int64_t jj = 0; jj < wk; ++jj) { hc.push_back(jj); hcd.push_back(jj); }
            const int64_t ldp = std::max<int64_t>(mloc, 1), ldh = std::max<int64_t>(nlc, 1);
            gather_idx(c, hr, hc, Hb.data(), n, hrd, hcd, Hl.data(), ldh);
            if (nlc > 0 && mloc > 0)
                lb::gemm(c, Op::NoTrans, Op::NoTrans, mloc, wk, nlc, T(1), ll.ptr, ll.ld, Hl.data(), ldh, T(0),
                         Pw.data(), ldp);
            else
                lb::set(c, Uplo::General, mloc, wk, T(0), T(0), Pw.data(), ldp);
            if (g.row().size() > 1) g.row().allreduce(Pw.data(), Pw.data(), size_t(ldp) * wk, scalar_type<T>(),
                                                      ReduceOp::Sum, loc, c.stream);
            LocalBlock<T> lw = Wm.local(loc, true);
            if (lw.n > 0 && lw.m > 0) {
                // my rows of W: G rows (rowg - kk) minus the reduced product
                const int64_t lr1 = lrow_of(Lm, k + 1);
                std::vector<int64_t> ri, rd, ci, cd;
                for (int64_t li = lr1; li < mloc; ++li) { ri.push_back(rowg[li] - kk); rd.push_back(li - lr1); }
                for (int64_t jj = 0; jj < wk; ++jj) { ci.push_back(jj); cd.push_back(jj); }
                gather_idx(c, ri, ci, G.data(), mk, rd, cd, lw.ptr, lw.ld);
                lb::add(c, Uplo::General, lw.m, wk, T(-1), Pw.data() + lr1, ldp, T(1), lw.ptr, lw.ld);
            }
            if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
        }
        // 7. distributed partial-pivoting LU of the panel
        Pivots pk;
        int64_t iinfo = getrf(Wm, pk, opts);
        if (iinfo && !info) info = ke + iinfo;
        pivots[k + 1] = pk.empty() ? std::vector<Pivot>() : pk[0];
        // tile-relative pivots of the single block -> absolute rows (>= ke)
        std::vector<int64_t> ip;
        for (int64_t t = 0; t < int64_t(pk.size()); ++t)
            for (auto const& pv : pk[t]) ip.push_back(ke + (t + pv.tileIndex()) * nb + pv.elementOffset());
        pivots[k + 1].clear();
        for (int64_t t = 0; t < int64_t(ip.size()) && t < w1; ++t) {
            const int64_t r = ip[t] - ke;
            pivots[k + 1].push_back(Pivot(r / nb, r % nb));
        }
        for (int64_t t = 0; t < int64_t(ip.size()) && t < w1; ++t) {
            const int64_t a = ke + t, b = ip[t];
            if (a != b) { std::swap(perm[a], perm[b]); pinv[perm[a]] = a; pinv[perm[b]] = b; }
        }
        // L(k+1:, 0:ke) rows follow the interchanges
        {
            Matrix<T> Lleft = Lm.sub(k + 1, nt - 1, 0, k);
            Pivots pk1(pk.begin(), pk.end());
            if (!pk1.empty()) pk1[0].resize(std::min<size_t>(pk1[0].size(), size_t(w1)));
            pk1.resize(1);
            internal::apply_pivots(pk1, BaseMatrix<T>(Wm), Lleft, target, true);
        }
        // L(k+1:, k+1) = the panel's unit-lower factor; U -> T(k+1, k) = U L(k,k)^{-H}
        {
            LocalBlock<T> lw = Wm.local(loc, false);
            LocalBlock<T> ll2 = Lm.local(loc, true);
            const int64_t lr1 = lrow_of(Lm, k + 1);
            lb::set(c, Uplo::General, nb, wk, T(0), T(0), Uw.data(), nb);
            if (lw.n > 0 && lw.m > 0) {
                const int64_t lc1 = lcol_of(Lm, k + 1);
                lb::copy2d(c, lw.m, w1, lw.ptr, lw.ld, ll2.ptr + lr1 + lc1 * ll2.ld, ll2.ld);
                if (Lm.srow_owner(k + 1) == g.myrow()) {
                    lb::copy(c, Uplo::Upper, Op::NoTrans, w1, wk, lw.ptr, lw.ld, Uw.data(), nb);
                    // unit lower diagonal block
                    T* Dk = ll2.ptr + lr1 + lc1 * ll2.ld;
                    if (w1 > 1) lb::set(c, Uplo::Upper, w1 - 1, w1 - 1, T(0), T(0), Dk + ll2.ld, ll2.ld);
                    lb::set(c, Uplo::General, 1, w1, T(1), T(1), Dk, ll2.ld + 1);
                }
            }
            sum_world(world, Uw.data(), size_t(nb) * wk, c);
            lb::trsm(c, Side::Right, Uplo::Lower, Op::ConjTrans, Diag::Unit, w1, wk, T(1), Lkk, nb, Uw.data(), nb);
            lb::copy2d(c, w1, wk, Uw.data(), nb, tsub(k), nb);
            if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
        }
    }
    // T -> the band matrix (kl = ku = nb): tiles (k, k), (k+1, k), (k, k+1)
    {
        trace::Block t2("aasen_band_T");
        Matrix<T> Tg(Tb);
        Tg.set_uplo(Uplo::General);
        set(T(0), T(0), Tg, opts);
        for (int64_t k = 0; k < nt; ++k)
            for (int64_t d = -1; d <= 1; ++d) {
                const int64_t i = k + (d > 0 ? 1 : 0), j = k + (d < 0 ? 1 : 0);
                if (i >= nt || j >= nt || !Tg.tileIsLocal(i, j)) continue;
                Tile<T> t = Tg.tile(i, j, loc);
                if (d == 0) lb::copy2d(c, t.mb, t.nb, tdiag(k), nb, t.data, t.stride);
                else if (d > 0) lb::copy2d(c, t.mb, t.nb, tsub(k), nb, t.data, t.stride);      // T(k+1, k)
                else lb::copy(c, Uplo::General, Op::ConjTrans, t.mb, t.nb, tsub(k), nb, t.data, t.stride);
            }
        if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
        Tg.storage()->modified(loc);
    }
    Tb.set_band(nb, nb);
    int64_t tinfo = gbtrf(Tb, pivots2, opts);
    if (!info && tinfo) info = tinfo;
    internal::finish_origin(Lm, opts);
    return internal::reduce_info(info, world);
}

template <typename T>
void hetrs(HermitianMatrix<T>& A, Pivots& pivots, BandMatrix<T>& Tb, Pivots& pivots2, Matrix<T>& B,
           Options const& opts) {
    trace::Block tb("hetrs_aasen");
    internal::DriverScope ds_;
    Target target = resolve_target(opts);
    Matrix<T> Lm(A);
    Lm.set_uplo(Uplo::General);
    TriangularMatrix<T> L(Uplo::Lower, Diag::Unit, Lm);
    internal::apply_pivots(pivots, BaseMatrix<T>(Lm), B, target, true);
    trsm(Side::Left, T(1), L, B, opts);
    gbtrs(Tb, pivots2, B, opts);
    trsm(Side::Left, T(1), TriangularMatrix<T>(conj_transpose(L)), B, opts);
    internal::apply_pivots(pivots, BaseMatrix<T>(Lm), B, target, false);
    internal::finish_origin(B, opts);
}

template <typename T>
int64_t hesv(HermitianMatrix<T>& A, Pivots& pivots, BandMatrix<T>& Tb, Pivots& pivots2, Matrix<T>& H, Matrix<T>& B,
             Options const& opts) {
    trace::Block tb("hesv_aasen");
    internal::DriverScope ds_;
    int64_t info = hetrf(A, pivots, Tb, pivots2, H, opts);
    if (info == 0) hetrs(A, pivots, Tb, pivots2, B, opts);
    return info;
}

#define SLATE_HE_INST(T)                                                                              \
    template int64_t hetrf<T>(HermitianMatrix<T>&, std::vector<int64_t>&, Options const&);           \
    template void hetrs<T>(HermitianMatrix<T> const&, std::vector<int64_t> const&, Matrix<T>&,       \
                           Options const&);                                                           \
    template int64_t hesv<T>(HermitianMatrix<T>&, std::vector<int64_t>&, Matrix<T>&, Options const&);           \
    template int64_t hetrf<T>(HermitianMatrix<T>&, Pivots&, BandMatrix<T>&, Pivots&, Matrix<T>&, Options const&); \
    template void hetrs<T>(HermitianMatrix<T>&, Pivots&, BandMatrix<T>&, Pivots&, Matrix<T>&, Options const&);    \
    template int64_t hesv<T>(HermitianMatrix<T>&, Pivots&, BandMatrix<T>&, Pivots&, Matrix<T>&, Matrix<T>&,      \
                             Options const&);

SLATE_HE_INST(float)
SLATE_HE_INST(double)
SLATE_HE_INST(std::complex<float>)
SLATE_HE_INST(std::complex<double>)

}  // namespace slate
