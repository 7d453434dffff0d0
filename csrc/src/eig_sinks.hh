// Shared stage-2 pieces of the eigen / SVD drivers: 1-D grids over a 2-D
// grid's processes and the row-local rotation sink (bdsqr / steqr rotations
// applied to each rank's rows of the vector matrices; reference
// src/bdsqr.cc, src/steqr2.cc keep the vectors distributed the same way).
#pragma once

#include "internal.hh"
#include "slate_amd/eig_host.hh"
#include "../kernels/kernels.hh"

#include <algorithm>

namespace slate {
namespace internal {

/// 1 x P grid over the processes of g (every row local: 1-D column layout)
inline GridPtr row_grid(GridPtr const& g) {
    if (g->p() == 1) return g;
    return std::make_shared<Grid>(1, g->size(), GridOrder::Col, g->world_ptr(), g->world_ptr(),
                                  std::make_shared<SelfComm>());
}

/// P x 1 grid over the processes of g (all columns local: 1-D row layout)
inline GridPtr col_grid(GridPtr const& g) {
    if (g->q() == 1) return g;
    return std::make_shared<Grid>(g->size(), 1, GridOrder::Col, g->world_ptr(), std::make_shared<SelfComm>(),
                                  g->world_ptr());
}

/// bdsqr transformations on the local rows of U and Vt (row layout: rows are
/// independent under column rotations, so no communication).  Device: QR
/// sweeps are batched kRotBatch at a time into step-ordered (c, s) tables
/// (pinned, double-buffered) and applied by the register-window wavefront
/// kernel while the host keeps iterating on (d, e); host: loops.
template <typename T>
struct RowRotSink : host::RotSink<real_type<T>> {
    using R = real_type<T>;
    using Rots = std::vector<host::PlaneRot<R>>;
    static constexpr int K = slate_amd::dev::kRotBatch;
    lb::Ctx c;
    int64_t n = 0;
    T* U = nullptr; int64_t ldu = 0, urows = 0;
    T* V = nullptr; int64_t ldv = 0, vrows = 0;
    size_t tsz = 0;                                // reals per table (one matrix)
    R* hb[2] = {nullptr, nullptr};
    Work<R> db[2];
    hipEvent_t ev[2] = {nullptr, nullptr};
    int cur = 0;
    std::vector<Rots> bu, bv;                      // the batch's sweeps

    RowRotSink(lb::Ctx const& c_, int64_t n_) : c(c_), n(n_) {
        if (c.dev()) {
            tsz = size_t(2 * K) * size_t(n + 2 * K);
            for (int b = 0; b < 2; ++b) {
                hb[b] = static_cast<R*>(device::malloc_host(sizeof(R) * 2 * tsz));
                db[b].resize(Target::Devices, 2 * tsz);
                ev[b] = device::event_get();
                slate_hip_call(hipEventRecord(ev[b], c.stream));
            }
        }
    }
    ~RowRotSink() override {
        if (c.dev()) {
            (void)hipStreamSynchronize(c.stream);
            for (int b = 0; b < 2; ++b) { device::free_host(hb[b]); device::event_put(ev[b]); }
        }
    }
    /// host twin of the rot_sweeps kernel (same table, same step order), so
    /// the CPU tests check the batching
    static void sweeps_host(int64_t rows, T* M, int64_t ld, int64_t p0, int64_t p1, R const* D) {
        if (p1 - p0 < 2) return;
        const int64_t tend = p1 - 2 + 2 * (K - 1);
        #pragma omp parallel for schedule(static) if (rows > 64)
        for (int64_t r = 0; r < rows; ++r) {
            T w[2 * K];
            for (int i = 0; i < 2 * K; ++i) w[i] = T(0);
            w[2 * K - 2] = M[r + p0 * ld];
            w[2 * K - 1] = (p0 + 1 < p1) ? M[r + (p0 + 1) * ld] : T(0);
            for (int64_t tau = p0; tau <= tend; ++tau) {
                R const* cs = D + 2 * K * (tau - p0);
                for (int q = 0; q < K; ++q) {
                    const R cc = cs[2 * q], sn = cs[2 * q + 1];
                    const T x = w[2 * K - 2 - 2 * q], y = w[2 * K - 1 - 2 * q];
                    w[2 * K - 2 - 2 * q] = x * cc - y * sn;
                    w[2 * K - 1 - 2 * q] = x * sn + y * cc;
                }
                const int64_t cr = tau - 2 * K + 2;
                if (cr >= p0) M[r + cr * ld] = w[0];
                for (int i = 0; i < 2 * K - 1; ++i) w[i] = w[i + 1];
                w[2 * K - 1] = (tau + 2 < p1) ? M[r + (tau + 2) * ld] : T(0);
            }
            M[r + (p1 - 1) * ld] = w[0];
        }
    }
    static std::pair<int64_t, int64_t> build(std::vector<Rots> const& b, R* D) {
        int64_t p0 = INT64_MAX, p1 = -1;
        for (auto const& rs : b)
            if (!rs.empty()) { p0 = std::min(p0, rs.front().i); p1 = std::max(p1, rs.back().i + 2); }
        if (p1 < 0) return {0, 0};
        const int64_t steps = p1 - p0 + 2 * K - 3;
        for (int64_t t = 0; t < steps; ++t)
            for (int q = 0; q < K; ++q) { D[2 * (t * K + q)] = R(1); D[2 * (t * K + q) + 1] = R(0); }
        for (size_t q = 0; q < b.size(); ++q)
            for (auto const& g : b[q]) {
                const int64_t t = g.i + 2 * int64_t(q) - p0;
                D[2 * (t * K + q)] = g.c;
                D[2 * (t * K + q) + 1] = g.s;
            }
        return {p0, p1};
    }
    void flush() {
        if (bu.empty()) return;
        if (!c.dev()) {
            std::vector<R> D(size_t(2 * K) * size_t(n + 2 * K));
            auto ru = build(bu, D.data());
            if (U) sweeps_host(urows, U, ldu, ru.first, ru.second, D.data());
            auto rv = build(bv, D.data());
            if (V) sweeps_host(vrows, V, ldv, rv.first, rv.second, D.data());
            recycle();
            return;
        }
        namespace kd_ = slate_amd::dev;
        R* Du = hb[cur];
        R* Dv = hb[cur] + tsz;
        std::pair<int64_t, int64_t> ru, rv;
        {
            trace::Block tb("bdsqr_rot_tables");
            ru = build(bu, Du);
            rv = build(bv, Dv);
        }
        const size_t su = size_t(std::max<int64_t>(ru.second - ru.first + 2 * K - 3, 0)) * 2 * K;
        const size_t sv = size_t(std::max<int64_t>(rv.second - rv.first + 2 * K - 3, 0)) * 2 * K;
        if (su) device::memcpy_async(db[cur].data(), Du, su * sizeof(R), c.stream);
        if (sv) device::memcpy_async(db[cur].data() + tsz, Dv, sv * sizeof(R), c.stream);
        kd_::rot_sweeps2(U && su ? urows : 0, kd_::dptr(U), ldu, ru.first, ru.second, db[cur].data(),
                         V && sv ? vrows : 0, kd_::dptr(V), ldv, rv.first, rv.second, db[cur].data() + tsz, c.stream);
        slate_hip_call(hipEventRecord(ev[cur], c.stream));
        cur ^= 1;
        recycle();
        trace::Block tw("bdsqr_rot_wait");
        slate_hip_call(hipEventSynchronize(ev[cur]));   // the other staging buffer is free again
    }
    void sweep(Rots& ru, Rots& rv) override {
        // take the sweep's rotations without copying (the caller clears its
        // vectors; spare ones keep their capacity for the next sweeps)
        bu.emplace_back();
        bv.emplace_back();
        if (!spare.empty()) { bu.back().swap(spare.back()); spare.pop_back(); }
        if (!spare.empty()) { bv.back().swap(spare.back()); spare.pop_back(); }
        bu.back().swap(ru);
        bv.back().swap(rv);
        if (int(bu.size()) == K) flush();
    }
    std::vector<Rots> spare;
    void recycle() {
        for (auto& r : bu) { r.clear(); spare.push_back(std::move(r)); }
        for (auto& r : bv) { r.clear(); spare.push_back(std::move(r)); }
        bu.clear();
        bv.clear();
    }
    void rot_u(int64_t a, int64_t b, R cc, R sn) override {
        if (!U) return;
        flush();
        if (!c.dev()) {
            T* x = U + a * ldu;
            T* y = U + b * ldu;
            for (int64_t r = 0; r < urows; ++r) {
                T p = x[r], q = y[r];
                x[r] = p * cc + q * sn;
                y[r] = q * cc - p * sn;
            }
            return;
        }
        flush();
        slate_amd::dev::rot_cols(urows, slate_amd::dev::dptr(U), ldu, a, b, cc, sn, c.stream);
    }
    void negate_v(int64_t k) override {
        if (!V) return;
        flush();
        lb::scale(c, Uplo::General, vrows, int64_t(1), R(-1), R(1), V + k * ldv, ldv);
    }
    void permute(std::vector<int64_t> const& perm) override {
        flush();
        auto pc = [&](T* M, int64_t ld, int64_t rows) {
            if (!M || rows <= 0) return;
            Work<T> tmp(c.dev() ? Target::Devices : Target::HostTask, size_t(rows) * n);
            if (c.dev()) {
                Work<int64_t> dp(Target::Devices, perm.size());
                device::memcpy_async(dp.data(), perm.data(), perm.size() * sizeof(int64_t), c.stream);
                slate_amd::dev::rbt_gather(false, false, n, rows, dp.data(), slate_amd::dev::dptr(M), ld,
                                           slate_amd::dev::dptr(tmp.data()), rows, c.stream);
                lb::copy2d(c, rows, n, tmp.data(), rows, M, ld);
                slate_hip_call(hipStreamSynchronize(c.stream));
            } else {
                for (int64_t i = 0; i < n; ++i)
                    for (int64_t r = 0; r < rows; ++r) tmp.data()[r + i * rows] = M[r + perm[i] * ld];
                for (int64_t i = 0; i < n; ++i)
                    for (int64_t r = 0; r < rows; ++r) M[r + i * ld] = tmp.data()[r + i * rows];
            }
        };
        pc(U, ldu, urows);
        pc(V, ldv, vrows);
    }
    void finish() {
        flush();
        if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
    }
};

}  // namespace internal
}  // namespace slate
