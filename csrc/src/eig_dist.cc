// Distributed stage 2 of the eigensolver: tridiagonal divide and conquer with
// the eigenvector matrix on the 2-D process grid (reference src/stedc.cc,
// stedc_solve.cc, stedc_merge.cc:171-190, stedc_z_vector.cc, stedc_sort.cc,
// stedc_deflate.cc, stedc_secular.cc) and the QR iteration with distributed
// eigenvector rows (reference src/steqr2.cc:60-74, {s,d,c,z}steqr2.f).
//
// stedc_dist.  The tridiagonal (d, e) is replicated (O(n)); Q lives ONLY in
// the distributed matrix (device instance on the device target).  The split
// tree follows Q's tiles: every leaf is one diagonal tile, solved by its owner
// on the host (nb x nb); every merge of two adjacent tile ranges
// [lo, mid) + [mid, hi):
//   * z = rows mid-1 / mid of Q over the block's columns: one world all-reduce
//     of n2 values;
//   * sort, deflation (tiny z, close pairs -> Givens rotations recorded, not
//     applied) on the host, replicated and deterministic: O(n2 log n2);
//   * secular roots and Gu-Eisenstat z on the device (one thread per root);
//   * the merge matrix M (Q_new = Q_old M, n2 x n2) built by every rank for
//     its OWN local entries only (kernels/stedc.hip);
//   * Q_new = [Q1 0; 0 Q2] M as two distributed MFMA GEMMs on the halves.
// No rank holds an n x n array on the host: per-rank host memory is O(n + nb^2).
//
// steqr2_dist.  Implicit QL (the host steqr's sweeps) on the replicated
// (d, e); every plane rotation acts on two columns of Z, i.e. row-wise, so
// with Z laid out by rows (P x 1 grid) each rank applies the rotations to its
// own rows with no communication -- on the device through the batched
// wavefront rotation kernel of bdsqr.
#include "internal.hh"
#include "eig_sinks.hh"
#include "slate_amd/eig_host.hh"
#include "slate_amd/secular.hh"
#include "../kernels/kernels.hh"

#include <algorithm>
#include <cmath>
#include <numeric>

namespace slate {
namespace internal {

namespace {

struct SplitNode { int64_t t0, tm, t1; double beta; };

/// post-order merge list of the tile-aligned bisection tree over tiles [t0, t1)
void split_tree(int64_t t0, int64_t t1, std::vector<SplitNode>& merges, std::vector<int64_t>& cuts) {
    if (t1 - t0 <= 1) return;
    const int64_t tm = (t0 + t1) / 2;
    split_tree(t0, tm, merges, cuts);
    split_tree(tm, t1, merges, cuts);
    merges.push_back({t0, tm, t1, 0.0});
    cuts.push_back(tm);
}

/// host twin of the device merge-matrix kernel (host target / tests)
template <typename R>
void merge_matrix_host(slate_amd::dev::StedcMerge const& m, std::vector<double> const& dd, std::vector<double> const& zh,
                       std::vector<double> const& tau, std::vector<int64_t> const& org, std::vector<int64_t> const& act,
                       std::vector<int64_t> const& defl, std::vector<int64_t> const& ord,
                       std::vector<int64_t> const& inv_perm, std::vector<int64_t> const& rab,
                       std::vector<double> const& rcs, int64_t ncols, R* M, int64_t ldm) {
    auto l2g_ = [](int64_t l, int64_t b, int64_t procs, int64_t rel) { return ((l / b) * procs + rel) * b + l % b; };
    #pragma omp parallel for schedule(dynamic, 4)
    for (int64_t lc = 0; lc < ncols; ++lc) {
        std::vector<double> vec(size_t(m.n2), 0.0);
        const int64_t jo = l2g_(m.lc0 + lc, m.nb, m.q, m.crel) - m.col_off;
        const int64_t r = ord[jo];
        if (r < m.k) {
            const double dr = dd[org[r]], tr = tau[r];
            double nrm = 0;
            for (int64_t i = 0; i < m.k; ++i) {
                const double u = zh[i] / ((dd[i] - dr) - tr);
                vec[act[i]] = u;
                nrm += u * u;
            }
            nrm = 1.0 / std::sqrt(nrm);
            for (int64_t i = 0; i < m.k; ++i) vec[act[i]] *= nrm;
        } else {
            vec[defl[r - m.k]] = 1.0;
        }
        for (int64_t t = m.nrot - 1; t >= 0; --t) {
            const int64_t x = rab[2 * t], y = rab[2 * t + 1];
            const double c = rcs[2 * t], sn = rcs[2 * t + 1], vx = vec[x], vy = vec[y];
            vec[x] = c * vx - sn * vy;
            vec[y] = sn * vx + c * vy;
        }
        for (int64_t lr = 0; lr < m.lrows; ++lr) {
            const int64_t src = l2g_(m.lr0 + lr, m.mb, m.p, m.rrel) - m.row_off;
            M[lr + lc * ldm] = R(vec[inv_perm[src]]);
        }
    }
}

/// secular roots + Gu-Eisenstat z on the host (same algorithm as the kernels)
void secular_host(int64_t k, double rho, std::vector<double> const& dd, std::vector<double> const& zz,
                  std::vector<int64_t>& org, std::vector<double>& tau, std::vector<double>& zh) {
    double znorm2 = 0;
    for (int64_t i = 0; i < k; ++i) znorm2 += zz[i] * zz[i];
    org.assign(k, 0); tau.assign(k, 0.0); zh.assign(k, 0.0);
    #pragma omp parallel for schedule(dynamic, 8) if (k > 64)
    for (int64_t j = 0; j < k; ++j) {
        int64_t o2 = j;
        tau[j] = secular::root<double>(k, j, rho, dd.data(), zz.data(), znorm2, &o2);
        org[j] = o2;
    }
    #pragma omp parallel for schedule(static) if (k > 256)
    for (int64_t i = 0; i < k; ++i) {
        auto lmd = [&](int64_t j) { return (dd[org[j]] - dd[i]) + tau[j]; };
        double pr = lmd(k - 1) / rho;
        for (int64_t j = 0; j < k - 1; ++j) pr *= lmd(j) / ((j < i) ? (dd[j] - dd[i]) : (dd[j + 1] - dd[i]));
        zh[i] = std::copysign(std::sqrt(std::abs(pr)), zz[i]);
    }
}

}  // namespace

template <typename R>
void stedc_dist(std::vector<R>& d, std::vector<R> const& e_in, Matrix<R>& Q, Options const& opts) {
    trace::Block tb("stedc_dist");
    internal::DriverScope ds_;
    const Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    const int64_t n = int64_t(d.size());
    slate_error_if_msg(Q.m() != n || Q.n() != n || Q.mb() != Q.nb() || !Q.aligned() || Q.op() != Op::NoTrans,
                       "stedc: Q must be an n x n NoTrans matrix with square tiles");
    if (n == 0) return;
    auto& g = *Q.grid();
    Comm& world = g.world();
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    std::vector<R> e(e_in.begin(), e_in.end());
    e.resize(std::max<int64_t>(n - 1, 0));
    const int64_t nt = Q.nt();
    std::vector<SplitNode> merges;
    std::vector<int64_t> cuts;
    split_tree(0, nt, merges, cuts);
    // tear at every cut (Cuppen): T = diag(T1, T2) + |beta| v v^T
    for (auto& nd : merges) {
        const int64_t mid = grow_of(Q, nd.tm);
        nd.beta = double(e[mid - 1]);
        const R rho0 = std::abs(e[mid - 1]);
        d[mid - 1] -= rho0;
        d[mid] -= rho0;
    }
    // ---- leaves: diagonal tiles, solved by their owners
    set(R(0), R(0), Q, opts);
    std::vector<R> dl(n, R(0));
    {
        trace::Block t2("stedc_leaves");
        Q.storage()->get(loc, true);
        for (int64_t t = 0; t < nt; ++t) {
            if (!Q.tileIsLocal(t, t)) continue;
            const int64_t r0 = grow_of(Q, t), nbt = Q.tileNb(t);
            std::vector<R> dt(d.begin() + r0, d.begin() + r0 + nbt), et(std::max<int64_t>(nbt - 1, 0));
            for (int64_t i = 0; i + 1 < nbt; ++i) et[i] = e[r0 + i];
            std::vector<R> Zt(size_t(nbt) * nbt);
            host::stedc<R>(nbt, dt.data(), et.data(), Zt.data(), nbt);
            Tile<R> tl = Q.tile(t, t, loc);
            if (c.dev()) {
                device::memcpy2d_async(tl.data, tl.stride * sizeof(R), Zt.data(), nbt * sizeof(R), nbt * sizeof(R), nbt,
                                       c.stream);
                slate_hip_call(hipStreamSynchronize(c.stream));
            } else {
                for (int64_t j = 0; j < nbt; ++j) std::copy(Zt.begin() + j * nbt, Zt.begin() + (j + 1) * nbt, tl.data + j * tl.stride);
            }
            std::copy(dt.begin(), dt.end(), dl.begin() + r0);
        }
        allreduce_host(world, dl.data(), size_t(n), ReduceOp::Sum);
        d = dl;
    }
    if (merges.empty()) return;
    Matrix<R> Qb = Q.emptyLike(), M = Q.emptyLike();
    Qb.insertLocalTiles(target);
    M.insertLocalTiles(target);
    auto& st = *Q.storage();
    Work<double> dvec, dscr;
    Work<int64_t> divec;
    for (auto const& nd : merges) {
        trace::Block t2("stedc_merge");
        const int64_t lo = grow_of(Q, nd.t0), mid = grow_of(Q, nd.tm), hi = grow_of(Q, nd.t1);
        const int64_t n1 = mid - lo, n2 = hi - lo;
        const double rho = 2.0 * std::abs(nd.beta), sgn = nd.beta < 0 ? -1.0 : 1.0;
        // ---- z: row mid-1 of Q over [lo, mid) and row mid over [mid, hi)
        std::vector<double> z(n2, 0.0);
        {
            trace::Block t3("stedc_m_z");
            LocalBlock<R> lq = Q.local(loc, false);
            auto grab = [&](int64_t grow, int64_t c0, int64_t c1, double scl) {
                if (st.row_owner(grow / st.mb) != g.myrow()) return;
                const int64_t lr = g2l(grow, st.mb, g.p());
                const int64_t lc0 = g2l_ceil(c0, st.nb, st.crel(), g.q()), lc1 = g2l_ceil(c1, st.nb, st.crel(), g.q());
                if (lc1 <= lc0) return;
                std::vector<R> row(lc1 - lc0);
                if (c.dev()) {
                    device::memcpy2d_async(row.data(), sizeof(R), lq.ptr + lr + lc0 * lq.ld, lq.ld * sizeof(R),
                                           sizeof(R), lc1 - lc0, c.stream);
                    slate_hip_call(hipStreamSynchronize(c.stream));
                } else {
                    for (int64_t t = lc0; t < lc1; ++t) row[t - lc0] = lq.ptr[lr + t * lq.ld];
                }
                for (int64_t t = lc0; t < lc1; ++t)
                    z[l2g(t, st.nb, st.crel(), g.q()) - lo] = scl * double(row[t - lc0]);
            };
            const double s2 = 1.0 / std::sqrt(2.0);
            grab(mid - 1, lo, mid, s2);
            grab(mid, mid, hi, sgn * s2);
            allreduce_host(world, z.data(), size_t(n2), ReduceOp::Sum);
        }
        // ---- sort (stable), deflation (rotations recorded)
        std::vector<int64_t> perm(n2);
        std::iota(perm.begin(), perm.end(), int64_t(0));
        std::stable_sort(perm.begin(), perm.end(), [&](int64_t a, int64_t b) { return d[lo + a] < d[lo + b]; });
        std::vector<double> Ds(n2), zs(n2);
        for (int64_t s = 0; s < n2; ++s) { Ds[s] = double(d[lo + perm[s]]); zs[s] = z[perm[s]]; }
        std::vector<char> defl_flag(n2, 0);
        std::vector<int64_t> rab;
        std::vector<double> rcs;
        {
            trace::Block t3("stedc_m_deflate");
            const double eps = std::numeric_limits<R>::epsilon();
            double dmax = 0, zmax = 0;
            for (int64_t j = 0; j < n2; ++j) { dmax = std::max(dmax, std::abs(Ds[j])); zmax = std::max(zmax, std::abs(zs[j])); }
            const double tol = 8.0 * eps * std::max(dmax, zmax * rho);
            for (int64_t j = 0; j < n2; ++j) defl_flag[j] = (rho * std::abs(zs[j]) <= tol) ? 1 : 0;
            int64_t last = -1;
            for (int64_t j = 0; j < n2; ++j) {
                if (defl_flag[j]) continue;
                if (last >= 0) {
                    const double t = std::hypot(zs[last], zs[j]);
                    const double cc = zs[j] / t, sn = -zs[last] / t;
                    if (std::abs((Ds[j] - Ds[last]) * cc * sn) <= tol) {
                        rab.push_back(last); rab.push_back(j);
                        rcs.push_back(cc); rcs.push_back(sn);
                        const double dlst = Ds[last], dj = Ds[j];
                        Ds[last] = dlst * cc * cc + dj * sn * sn;
                        Ds[j] = dlst * sn * sn + dj * cc * cc;
                        zs[j] = t;
                        zs[last] = 0;
                        defl_flag[last] = 1;
                    }
                }
                last = j;
            }
        }
        std::vector<int64_t> act, defl;
        for (int64_t j = 0; j < n2; ++j) (defl_flag[j] ? defl : act).push_back(j);
        std::sort(act.begin(), act.end(), [&](int64_t a, int64_t b) { return Ds[a] < Ds[b]; });
        const int64_t k = int64_t(act.size());
        std::vector<double> dd(k), zz(k);
        for (int64_t i = 0; i < k; ++i) { dd[i] = Ds[act[i]]; zz[i] = zs[act[i]]; }
        // ---- secular roots (device or host), eigenvalues, output order
        std::vector<int64_t> org;
        std::vector<double> tau, zh;
        const bool dev = c.dev();
        // device vector block: dd k | zz k | tau k | zh k | rcs 2 nrot ; ints: org k | act k | defl n2-k | ord n2 | inv n2 | rab 2 nrot
        const int64_t nrot = int64_t(rcs.size()) / 2;
        trace::Block t3s("stedc_m_secular");
        if (dev) {
            dvec.resize(Target::Devices, size_t(4 * k + 2 * nrot + 1));
            divec.resize(Target::Devices, size_t(2 * k + 3 * n2 + 2 * nrot + 1));
            double znorm2 = 0;
            for (int64_t i = 0; i < k; ++i) znorm2 += zz[i] * zz[i];
            device::memcpy_async(dvec.data(), dd.data(), k * sizeof(double), c.stream);
            device::memcpy_async(dvec.data() + k, zz.data(), k * sizeof(double), c.stream);
            slate_amd::dev::secular_roots(k, rho, dvec.data(), dvec.data() + k, znorm2, divec.data(), dvec.data() + 2 * k,
                                          c.stream);
            slate_amd::dev::gu_eisenstat(k, rho, dvec.data(), dvec.data() + k, divec.data(), dvec.data() + 2 * k,
                                         dvec.data() + 3 * k, c.stream);
            org.resize(k);
            tau.resize(k);
            device::memcpy_async(org.data(), divec.data(), k * sizeof(int64_t), c.stream);
            device::memcpy_async(tau.data(), dvec.data() + 2 * k, k * sizeof(double), c.stream);
            slate_hip_call(hipStreamSynchronize(c.stream));
        } else {
            secular_host(k, rho, dd, zz, org, tau, zh);
        }
        t3s.end();
        std::vector<double> lam(n2);
        for (int64_t r = 0; r < k; ++r) lam[r] = dd[org[r]] + tau[r];
        for (int64_t cdx = 0; cdx < n2 - k; ++cdx) lam[k + cdx] = Ds[defl[cdx]];
        std::vector<int64_t> ord(n2), inv_perm(n2);
        std::iota(ord.begin(), ord.end(), int64_t(0));
        std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return lam[a] < lam[b]; });
        for (int64_t s = 0; s < n2; ++s) inv_perm[perm[s]] = s;
        // ---- merge matrix: my local entries of the n2 x n2 block
        trace::Block t3m("stedc_m_matrix");
        Matrix<R> Mb = M.sub(nd.t0, nd.t1 - 1, nd.t0, nd.t1 - 1);
        LocalBlock<R> lm = Mb.local(loc, true);
        slate_amd::dev::StedcMerge mg;
        mg.n2 = n2; mg.k = k; mg.nrot = nrot;
        mg.lrows = lm.m; mg.mb = st.mb; mg.p = g.p(); mg.rrel = st.rrel(); mg.row_off = lo;
        mg.nb = st.nb; mg.q = g.q(); mg.crel = st.crel(); mg.col_off = lo;
        mg.lr0 = Mb.lrow_begin(); mg.lc0 = Mb.lcol_begin();
        if (dev) {
            int64_t* iv = divec.data();
            device::memcpy_async(iv + k, act.data(), k * sizeof(int64_t), c.stream);
            if (n2 > k) device::memcpy_async(iv + 2 * k, defl.data(), (n2 - k) * sizeof(int64_t), c.stream);
            device::memcpy_async(iv + k + n2, ord.data(), n2 * sizeof(int64_t), c.stream);
            device::memcpy_async(iv + k + 2 * n2, inv_perm.data(), n2 * sizeof(int64_t), c.stream);
            if (nrot) {
                device::memcpy_async(iv + k + 3 * n2, rab.data(), 2 * nrot * sizeof(int64_t), c.stream);
                device::memcpy_async(dvec.data() + 4 * k, rcs.data(), 2 * nrot * sizeof(double), c.stream);
            }
            mg.dd = dvec.data(); mg.zh = dvec.data() + 3 * k; mg.tau = dvec.data() + 2 * k;
            mg.org = iv; mg.act = iv + k; mg.defl = iv + 2 * k; mg.ord = iv + k + n2; mg.inv_perm = iv + k + 2 * n2;
            mg.rot_ab = iv + k + 3 * n2; mg.rot_cs = dvec.data() + 4 * k;
            // columns in batches: scratch of batch x n2 reals
            const int64_t batch = std::max<int64_t>(1, std::min<int64_t>(lm.n, int64_t(256 << 20) / (8 * std::max<int64_t>(n2, 1))));
            dscr.resize(Target::Devices, size_t(batch) * n2);
            for (int64_t c0 = 0; c0 < lm.n; c0 += batch)
                slate_amd::dev::merge_matrix<R>(mg, c0, std::min(batch, lm.n - c0), lm.ptr, lm.ld, dscr.data(), c.stream);
            slate_hip_call(hipStreamSynchronize(c.stream));
        } else {
            merge_matrix_host<R>(mg, dd, zh, tau, org, act, defl, ord, inv_perm, rab, rcs, lm.n, lm.ptr, lm.ld);
        }
        t3m.end();
        // ---- Q_new = [Q1 0; 0 Q2] M  (two GEMMs on the halves), back into Q
        {
            trace::Block t3("stedc_m_gemm");
            Matrix<R> Q1 = Q.sub(nd.t0, nd.tm - 1, nd.t0, nd.tm - 1), Q2 = Q.sub(nd.tm, nd.t1 - 1, nd.tm, nd.t1 - 1);
            Matrix<R> Mt = M.sub(nd.t0, nd.tm - 1, nd.t0, nd.t1 - 1), Mbot = M.sub(nd.tm, nd.t1 - 1, nd.t0, nd.t1 - 1);
            Matrix<R> Ct = Qb.sub(nd.t0, nd.tm - 1, nd.t0, nd.t1 - 1), Cb = Qb.sub(nd.tm, nd.t1 - 1, nd.t0, nd.t1 - 1);
            gemm(R(1), Q1, Mt, R(0), Ct, opts);
            gemm(R(1), Q2, Mbot, R(0), Cb, opts);
            Matrix<R> Qd = Q.sub(nd.t0, nd.t1 - 1, nd.t0, nd.t1 - 1), Qs = Qb.sub(nd.t0, nd.t1 - 1, nd.t0, nd.t1 - 1);
            slate::copy<R, R>(Qs, Qd, opts);
        }
        for (int64_t jo = 0; jo < n2; ++jo) d[lo + jo] = R(lam[ord[jo]]);
        (void)n1;
    }
}

//------------------------------------------------------------------------------
namespace {

/// Rotations of the QL sweeps applied to the local rows of Z (rows are
/// independent under column rotations).  QL sweeps run with i descending; on
/// the column-reversed Z (column j' = n-1-j: base Z + (n-1) ld, leading
/// dimension -ld) they are ASCENDING sweeps of the rotations (n-2-i, c, -s),
/// which the bdsqr row sink batches into its wavefront tables -- the device
/// kernel and its host twin alike, so the CPU tests check the reflection.
template <typename T>
struct QlRowSink : host::RotSink<real_type<T>> {
    using R = real_type<T>;
    lb::Ctx c;
    int64_t n, rows, ld;
    T* Z;
    RowRotSink<T> rs;
    std::vector<host::PlaneRot<R>> none;
    QlRowSink(lb::Ctx const& c_, int64_t n_, T* Z_, int64_t ld_, int64_t rows_)
        : c(c_), n(n_), rows(rows_), ld(ld_), Z(Z_), rs(c_, n_) {
        rs.U = rows > 0 ? Z + (n - 1) * ld : nullptr;
        rs.ldu = -ld;
        rs.urows = rows;
    }
    void flush() { rs.finish(); }
    void sweep(std::vector<host::PlaneRot<R>>& ru, std::vector<host::PlaneRot<R>>&) override {
        std::vector<host::PlaneRot<R>> asc(ru.size());
        for (size_t t = 0; t < ru.size(); ++t) asc[t] = {n - 2 - ru[t].i, ru[t].c, -ru[t].s};
        std::sort(asc.begin(), asc.end(), [](auto const& a, auto const& b) { return a.i < b.i; });
        none.clear();
        rs.sweep(asc, none);
    }
    void rot_u(int64_t, int64_t, R, R) override { slate_error("steqr2: unexpected rotation"); }
    void negate_v(int64_t) override {}
    void permute(std::vector<int64_t> const& perm) override {
        flush();
        if (rows <= 0) return;
        Work<T> tmp(c.dev() ? Target::Devices : Target::HostTask, size_t(rows) * n);
        if (c.dev()) {
            Work<int64_t> dp(Target::Devices, perm.size());
            device::memcpy_async(dp.data(), perm.data(), perm.size() * sizeof(int64_t), c.stream);
            slate_amd::dev::rbt_gather(false, false, n, rows, dp.data(), slate_amd::dev::dptr(Z), ld,
                                       slate_amd::dev::dptr(tmp.data()), rows, c.stream);
            lb::copy2d(c, rows, n, tmp.data(), rows, Z, ld);
            slate_hip_call(hipStreamSynchronize(c.stream));
            return;
        }
        for (int64_t i = 0; i < n; ++i)
            for (int64_t r = 0; r < rows; ++r) tmp.data()[r + i * rows] = Z[r + perm[i] * ld];
        for (int64_t i = 0; i < n; ++i)
            for (int64_t r = 0; r < rows; ++r) Z[r + i * ld] = tmp.data()[r + i * rows];
    }
};

}  // namespace

template <typename T>
int64_t steqr2_dist(std::vector<real_type<T>>& d, std::vector<real_type<T>>& e_in, Matrix<T>& Z, Options const& opts) {
    trace::Block tb("steqr2_dist");
    internal::DriverScope ds_;
    using R = real_type<T>;
    const Target target = resolve_target(opts);
    const Loc loc = loc_of(target);
    const int64_t n = int64_t(d.size());
    if (n == 0) return 0;
    std::vector<R> e(e_in.begin(), e_in.end());
    e.resize(std::max<int64_t>(n - 1, 0));
    // Z by rows (P x 1 grid): every rank owns whole rows
    auto g = Z.grid();
    GridPtr gr = col_grid(g);
    const bool rowlayout = (g->q() == 1 && Z.op() == Op::NoTrans && Z.aligned());
    Matrix<T> Zr = rowlayout ? Z : Matrix<T>(Z.m(), Z.n(), Z.mb(), std::max<int64_t>(Z.n(), 1), gr);
    if (!rowlayout) {
        Zr.insertLocalTiles(target);
        slate::copy<T, T>(Z, Zr, opts);
    }
    LocalBlock<T> lz = Zr.local(loc, true);
    lb::Ctx c = target == Target::Devices ? lb::Ctx::device(0) : lb::Ctx::host();
    QlRowSink<T> sink(c, n, lz.ptr, lz.ld, lz.m);
    int64_t info = host::steqr_core<R>(n, d.data(), e.data(), &sink);
    sink.flush();
    if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
    if (!rowlayout) slate::copy<T, T>(Zr, Z, opts);
    else internal::finish_origin(Z, opts);
    return info;
}

template void stedc_dist<float>(std::vector<float>&, std::vector<float> const&, Matrix<float>&, Options const&);
template void stedc_dist<double>(std::vector<double>&, std::vector<double> const&, Matrix<double>&, Options const&);
template int64_t steqr2_dist<float>(std::vector<float>&, std::vector<float>&, Matrix<float>&, Options const&);
template int64_t steqr2_dist<double>(std::vector<double>&, std::vector<double>&, Matrix<double>&, Options const&);
template int64_t steqr2_dist<std::complex<float>>(std::vector<float>&, std::vector<float>&,
                                                  Matrix<std::complex<float>>&, Options const&);
template int64_t steqr2_dist<std::complex<double>>(std::vector<double>&, std::vector<double>&,
                                                   Matrix<std::complex<double>>&, Options const&);

}  // namespace internal
}  // namespace slate
