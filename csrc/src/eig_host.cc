// Host stages of the two-stage eigen/SVD reductions (see eig_host.hh).
#include "slate_amd/eig_host.hh"
#include "slate_amd/host_blas.hh"
#include "slate_amd/secular.hh"
#include "slate_amd/exception.hh"

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <complex>
#include <limits>
#include <numeric>
#include <atomic>
#include <memory>
#include <immintrin.h>
#include <thread>
#include <omp.h>

namespace slate {
namespace host {

namespace {

/// sqrt(a^2 + b^2) without hypot's scaling when the squares are safely in
/// range (bdsqr's host loop makes two per rotation and is the SVD's critical
/// path: n = 4096 bidiagonal 1.17 -> 0.80-0.85 s); falls back to std::hypot
/// near under- / overflow.
template <typename R>
inline R fast_hypot(R a, R b) {
    const R s = a * a + b * b;
    constexpr R lo = std::numeric_limits<R>::min() * R(1 << 20);
    constexpr R hi = std::numeric_limits<R>::max() / R(1 << 20);
    if (s > lo && s < hi) return std::sqrt(s);
    return std::hypot(a, b);
}

// Wait for a pipelined sweep's progress counter: a short pause spin first
// (the lag between sweeps is a few microseconds of work), sched_yield only
// when the producer is really behind.
inline void wait_progress(std::atomic<int64_t> const& p, int64_t want) {
    for (int spin = 0; p.load(std::memory_order_acquire) < want; ++spin) {
        if (spin < 256) _mm_pause();
        else std::this_thread::yield();
    }
}

/// Sweeps per thread of the pipelined bulge chases (SLATE_SWEEP_GROUP;
/// n = 8192, 16 threads: hb2st 585 / 517 / 584 ms and tb2bd 934 / 690 / 979
/// ms at 1 / 2 / 4, profiles/r4_sweep_group.txt).
int64_t sweep_group() {
    static const int64_t g = [] {
        const char* s = std::getenv("SLATE_SWEEP_GROUP");
        const long v = s ? std::atol(s) : 0;
        return int64_t(v > 0 ? std::min(v, 64L) : 2);
    }();
    return g;
}

/// The bulge chases' pipeline: nsw sweeps, sweep j's step t may run once
/// sweep j-1 has finished kLag steps more (progress counters).  Each thread
/// takes GROUPS of G consecutive sweeps and advances them as a wavefront
/// (sweep g of the group kLag steps behind sweep g-1): step t of sweep j+1
/// rewrites the window sweep j left kLag steps earlier, so with the two on
/// one core the window is still in its L2, where handing every sweep to the
/// next thread (the previous scheme) moved the whole window between cores
/// each step -- 3x the single-thread cost of a step at 8 threads.  Only a
/// group's first sweep waits on another thread.  init(j) -> state;
/// step(state&, tid) -> false once the sweep has ended.
template <typename Init, typename Step>
void pipelined_sweeps(int64_t nsw, int64_t kLag, bool par, Init init, Step step) {
    using State = decltype(init(int64_t(0)));
    constexpr int64_t kDone = std::numeric_limits<int64_t>::max();
    std::unique_ptr<std::atomic<int64_t>[]> prog(new std::atomic<int64_t>[std::max<int64_t>(nsw, 1)]);
    for (int64_t j = 0; j < nsw; ++j) prog[j].store(0, std::memory_order_relaxed);
    const int64_t G = sweep_group();
    const int64_t ngroups = (nsw + G - 1) / G;
    #pragma omp parallel if (par)
    {
        const int nth = par ? omp_get_num_threads() : 1, tid = par ? omp_get_thread_num() : 0;
        std::vector<State> st;
        std::vector<int64_t> t;
        std::vector<char> done;
        // round-robin groups: the sweep before a group is always owned by
        // another running thread (or finished earlier by this one)
        for (int64_t gi = tid; gi < ngroups; gi += nth) {
            const int64_t j0 = gi * G, ng = std::min(G, nsw - j0);
            st.clear();
            for (int64_t g = 0; g < ng; ++g) st.push_back(init(j0 + g));
            t.assign(size_t(ng), 0);
            done.assign(size_t(ng), 0);
            int64_t left = ng;
            while (left > 0) {
                // latest sweep first: the next group waits on the last one,
                // so it gets started after ~kLag steps per sweep of this
                // group rather than kLag ROUNDS of all of them
                bool moved = false;
                for (int64_t g = ng - 1; g >= 0 && !moved; --g) {
                    if (done[g]) continue;
                    const int64_t j = j0 + g;
                    if (j > 0 && prog[j - 1].load(std::memory_order_acquire) < t[g] + kLag) continue;
                    const bool more = step(st[g], tid);
                    ++t[g];
                    moved = true;
                    if (more) {
                        prog[j].store(t[g], std::memory_order_release);
                    } else {
                        prog[j].store(kDone, std::memory_order_release);
                        done[g] = 1;
                        --left;
                    }
                }
                if (!moved) {
                    int64_t g = 0;
                    while (done[g]) ++g;
                    wait_progress(prog[j0 + g - 1], t[g] + kLag);
                }
            }
        }
    }
}

template <typename T> inline T cj(T x) { return x; }
template <typename R> inline std::complex<R> cj(std::complex<R> x) { return std::conj(x); }

/// sum_i conj(v[i]) x[i] with 16 independent partial sums: without
/// -ffast-math the compiler keeps a plain `s += ...` loop as ONE dependent
/// FMA chain (4 cycles a term), which made the bulge chase's dot products --
/// tb2bd's left update, hb2st's hemv -- latency-bound at ~1 GFLOP/s (tb2bd
/// 24 -> 9 us a step single-threaded with the split sums).
template <typename T>
inline T dotc(int64_t L, const T* __restrict__ v, const T* __restrict__ x) {
    constexpr int U = 16;
    T acc[U] = {};
    int64_t i = 0;
    for (; i + U <= L; i += U)
        for (int u = 0; u < U; ++u) acc[u] += cj(v[i + u]) * x[i + u];
    T s = T(0);
    for (; i < L; ++i) s += cj(v[i]) * x[i];
    for (int u = 0; u < U / 2; ++u) acc[u] += acc[u + U / 2];
    for (int u = 0; u < U / 4; ++u) acc[u] += acc[u + U / 4];
    return s + ((acc[0] + acc[2]) + (acc[1] + acc[3]));
}

/// One Givens rotation (c, s) on columns (i, i+1) of a row-major-agnostic
/// column-major matrix: [x y] <- [c*x - s*y, s*x + c*y].
template <typename R>
struct Rot { int64_t i; R c, s; };

/// Apply a recorded sequence of rotations to the rows of Z in parallel
/// (every row is independent; the sequence order is preserved per row).
template <typename R, typename T>
void apply_rots(std::vector<Rot<R>> const& rots, T* Z, int64_t ldz, int64_t zrows) {
    if (rots.empty() || Z == nullptr || zrows <= 0) return;
    const int64_t RB = 64;
    #pragma omp parallel for schedule(static) if (zrows * int64_t(rots.size()) > 32768)
    for (int64_t r0 = 0; r0 < zrows; r0 += RB) {
        int64_t r1 = std::min(zrows, r0 + RB);
        for (auto const& g : rots) {
            T* x = Z + g.i * ldz;
            T* y = Z + (g.i + 1) * ldz;
            for (int64_t k = r0; k < r1; ++k) {
                T a = x[k], b = y[k];
                x[k] = g.c * a - g.s * b;
                y[k] = g.s * a + g.c * b;
            }
        }
    }
}

}  // namespace

//------------------------------------------------------------------------------
template <typename T>
void Reflectors<T>::apply_left(bool trans, int64_t ncols, T* C, int64_t ldc) const {
    const int64_t K = int64_t(tau.size());
    if (K == 0 || ncols <= 0) return;
    const int64_t CB = 16;
    #pragma omp parallel for schedule(dynamic)
    for (int64_t c0 = 0; c0 < ncols; c0 += CB) {
        int64_t c1 = std::min(ncols, c0 + CB);
        for (int64_t t = 0; t < K; ++t) {
            int64_t k = trans ? t : K - 1 - t;
            T tk = trans ? cj(tau[k]) : tau[k];
            if (tk == T(0)) continue;
            const T* vk = v.data() + voff[k];
            int64_t o = off[k], L = len[k];
            for (int64_t j = c0; j < c1; ++j) {
                T* cc = C + o + j * ldc;
                T s = dotc(L, vk, cc) * tk;
                for (int64_t i = 0; i < L; ++i) cc[i] -= vk[i] * s;
            }
        }
    }
}

//------------------------------------------------------------------------------
// hb2st: sweeps j = 0..n-3; each annihilates column j below the subdiagonal
// with a reflector on rows [j+1, j+kd] and chases the bulge down the band by
// annihilating its first column kd rows further each time.
template <typename T>
void hb2st(int64_t n, int64_t kd, T* A, int64_t lda, std::vector<real_type<T>>& d, std::vector<real_type<T>>& e,
           Reflectors<T>& Q, std::vector<T>& phase) {
    using R = real_type<T>;
    auto a = [&](int64_t i, int64_t j) -> T& { return A[i + j * lda]; };
    const int64_t b = std::max<int64_t>(kd, 1);
    // per-thread scratch: v (reflector), w (dot products / the rank-2 vector)
    // H^H A H with H = I - tau v v^H on rows / columns J = [s0, s0 + L),
    // maintaining the LOWER triangle only (every later read -- the bulge
    // column, the next windows, d / e -- is a lower entry), which halves the
    // flops and the bytes of a step against updating both triangles:
    //   (d) rows J, columns (k, s0): left update only;
    //   (b) the J x J block: x = tau A_JJ v (lower hemv), w = x - conj(tau)/2
    //       (v^H x) v, A_JJ -= v w^H + w v^H (lower part);
    //   (c) rows (s0 + L - 1, s0 + L - 1 + b], columns J: right update only.
    // The upper triangle of the window is left stale (never read again).
    auto two_sided = [&](int64_t k, int64_t s0, int64_t L, T tau, const T* __restrict__ v, T* __restrict__ w) {
        const T ctau = cj(tau);
        // (d)
        for (int64_t c = k + 1; c < s0; ++c) {
            T* __restrict__ col = &a(s0, c);
            const T sum = dotc(L, v, col) * ctau;
            for (int64_t i = 0; i < L; ++i) col[i] -= v[i] * sum;
        }
        // (b)
        std::fill(w, w + L, T(0));
        for (int64_t l = 0; l < L; ++l) {
            const T* __restrict__ col = &a(s0, s0 + l);
            const T vl = v[l];
            for (int64_t i = l + 1; i < L; ++i) w[i] += col[i] * vl;
            // sum_i conj(col[i]) v[i] = conj(sum_i conj(v[i]) col[i])
            w[l] += T(std::real(col[l])) * vl + cj(dotc(L - l - 1, v + l + 1, col + l + 1));
        }
        for (int64_t i = 0; i < L; ++i) w[i] *= tau;
        const T vx = dotc(L, v, w);
        const T alpha = T(-0.5) * ctau * vx;
        for (int64_t i = 0; i < L; ++i) w[i] += alpha * v[i];
        for (int64_t l = 0; l < L; ++l) {
            T* __restrict__ col = &a(s0, s0 + l);
            const T cwl = cj(w[l]), cvl = cj(v[l]);
            for (int64_t i = l; i < L; ++i) col[i] -= v[i] * cwl + w[i] * cvl;
            if constexpr (is_complex_v<T>) col[l] = T(std::real(col[l]));
        }
        // (c)
        const int64_t r0 = s0 + L, r1 = std::min<int64_t>(n - 1, s0 + L - 1 + b);
        const int64_t nr = r1 - r0 + 1;
        if (nr <= 0) return;
        T* __restrict__ wr = w + L;
        std::fill(wr, wr + nr, T(0));
        for (int64_t l = 0; l < L; ++l) {
            const T* __restrict__ col = &a(r0, s0 + l);
            const T vl = v[l];
            for (int64_t r = 0; r < nr; ++r) wr[r] += col[r] * vl;
        }
        for (int64_t l = 0; l < L; ++l) {
            T* __restrict__ col = &a(r0, s0 + l);
            const T f = tau * cj(v[l]);
            for (int64_t r = 0; r < nr; ++r) col[r] -= wr[r] * f;
        }
    };
    // Sweeps are pipelined over threads (the reference's hb2st.cc runs its
    // bulge-chasing sweeps as OpenMP tasks the same way).  Step t of sweep j
    // (lower triangle only) touches rows [s0, s0 + 2b) x columns [s0 - b,
    // s0 + b) with s0 = j + 1 + t b; sweep j-1's step t' sits at s0 - 1 +
    // (t' - t) b, so the two rectangles share elements only for t' <= t + 2
    // (at t' = t + 2: its bulge column is row block (c) of this step).  Step t
    // therefore runs once sweep j-1 has finished its steps 0..t+2, and sweep
    // j-1's later steps cannot reach back into it.  Reflectors are collected
    // per sweep and concatenated in sweep order: reflectors of different
    // sweeps that ran out of order act on disjoint rows and commute.
    const int64_t nsw = (b > 1 && n > 2) ? n - 2 : 0;
    constexpr int64_t kLag = 3;
    std::vector<Reflectors<T>> Qs(nsw);
    struct St { int64_t j, k, s0, s1; };
    const bool par = nsw >= 64 && n >= 8 * b;
    std::vector<std::vector<T>> vs(size_t(par ? omp_get_max_threads() : 1)), ws(vs.size());
    for (auto& x : vs) x.resize(size_t(b + 1));
    for (auto& x : ws) x.resize(size_t(n));
    pipelined_sweeps(nsw, kLag, par,
        [&](int64_t j) { return St{j, j, j + 1, std::min(j + b, n - 1)}; },
        [&](St& q, int tid) {
            T* v = vs[tid].data();
            T* w = ws[tid].data();
            const int64_t L = q.s1 - q.s0 + 1;
            if (L < 2) return false;
            T alpha = a(q.s0, q.k);
            for (int64_t i = 1; i < L; ++i) v[i] = a(q.s0 + i, q.k);
            T tau;
            larfg(L, alpha, v + 1, 1, tau);
            v[0] = T(1);
            a(q.s0, q.k) = alpha;
            for (int64_t i = 1; i < L; ++i) a(q.s0 + i, q.k) = T(0);
            if (tau != T(0)) {
                two_sided(q.k, q.s0, L, tau, v, w);
                Qs[q.j].push(q.s0, L, tau, v, q.j);
            }
            // next bulge: column s0 below its band
            const int64_t ns0 = q.s0 + b, ns1 = std::min(q.s1 + b, n - 1);
            if (ns0 >= n - 1 || ns1 <= ns0) return false;
            q.k = q.s0; q.s0 = ns0; q.s1 = ns1;
            return true;
        });
    for (auto& q : Qs) {
        for (size_t r = 0; r < q.size(); ++r) Q.push(q.off[r], q.len[r], q.tau[r], q.v.data() + q.voff[r], q.tag[r]);
        q = Reflectors<T>();
    }
    d.assign(n, R(0));
    e.assign(std::max<int64_t>(n - 1, 0), R(0));
    phase.assign(n, T(1));
    for (int64_t i = 0; i < n; ++i) d[i] = std::real(a(i, i));
    for (int64_t i = 0; i + 1 < n; ++i) {
        T t = a(i + 1, i);
        R at = std::abs(t);
        e[i] = at;
        phase[i + 1] = at > R(0) ? phase[i] * t / T(at) : phase[i];
    }
}

//------------------------------------------------------------------------------
// tb2bd: sweeps j = 0..n-2: a right reflector on columns [j+1, j+kd] clears
// row j beyond the superdiagonal; the bulge below the diagonal is chased with
// alternating left (column) and right (row) reflectors.
template <typename T>
void tb2bd(int64_t m, int64_t n, int64_t kd, T* A, int64_t lda, std::vector<real_type<T>>& d,
           std::vector<real_type<T>>& e, Reflectors<T>& QU, Reflectors<T>& QV, std::vector<T>& pu,
           std::vector<T>& pv) {
    using R = real_type<T>;
    auto a = [&](int64_t i, int64_t j) -> T& { return A[i + j * lda]; };
    const int64_t b = std::max<int64_t>(kd, 1);
    // v (reflector) and w (window dot products) are per-thread scratch
    auto right = [&](int64_t r, int64_t c0, int64_t L, T tau, const T* v, T* w) {
        // rows in window (skip r): A[row, J] = A[row, J] H, column-oriented
        // (contiguous inner loops; the row-wise form strides by lda)
        // rows with nonzeros in columns [c0, c0 + L): the band rows
        // [c0 - b, c0 + L) (earlier rows are bidiagonal already, and the
        // previous sweep's bulge is kLag steps further down)
        int64_t w0 = std::max<int64_t>(0, c0 - b), w1 = std::min<int64_t>(m - 1, c0 + L - 1);
        const int64_t nr = w1 - w0 + 1;
        if (nr <= 0) return;
        // four columns per pass: w is loaded / stored once per four
        // column FMAs instead of once per column (the passes were
        // load/store-bound on w)
        std::fill(w, w + nr, T(0));
        int64_t t = 0;
        for (; t + 4 <= L; t += 4) {
            const T* __restrict__ x0 = &a(w0, c0 + t);
            const T* __restrict__ x1 = x0 + lda;
            const T* __restrict__ x2 = x1 + lda;
            const T* __restrict__ x3 = x2 + lda;
            const T v0 = v[t], v1 = v[t + 1], v2 = v[t + 2], v3 = v[t + 3];
            for (int64_t i = 0; i < nr; ++i) w[i] += (x0[i] * v0 + x1[i] * v1) + (x2[i] * v2 + x3[i] * v3);
        }
        for (; t < L; ++t) {
            const T* __restrict__ col = &a(w0, c0 + t);
            const T vt = v[t];
            for (int64_t i = 0; i < nr; ++i) w[i] += col[i] * vt;
        }
        const bool skip = (r >= w0 && r <= w1);
        T keep[4];
        for (t = 0; t < L; t += 4) {
            const int64_t nt = std::min<int64_t>(4, L - t);
            if (skip) for (int64_t u = 0; u < nt; ++u) keep[u] = a(r, c0 + t + u);  // row r is excluded
            if (nt == 4) {
                T* __restrict__ x0 = &a(w0, c0 + t);
                T* __restrict__ x1 = x0 + lda;
                T* __restrict__ x2 = x1 + lda;
                T* __restrict__ x3 = x2 + lda;
                const T f0 = tau * cj(v[t]), f1 = tau * cj(v[t + 1]), f2 = tau * cj(v[t + 2]), f3 = tau * cj(v[t + 3]);
                for (int64_t i = 0; i < nr; ++i) {
                    const T wi = w[i];
                    x0[i] -= wi * f0;
                    x1[i] -= wi * f1;
                    x2[i] -= wi * f2;
                    x3[i] -= wi * f3;
                }
            } else {
                for (int64_t u = 0; u < nt; ++u) {
                    T* __restrict__ col = &a(w0, c0 + t + u);
                    const T f = tau * cj(v[t + u]);
                    for (int64_t i = 0; i < nr; ++i) col[i] -= w[i] * f;
                }
            }
            if (skip) for (int64_t u = 0; u < nt; ++u) a(r, c0 + t + u) = keep[u];
        }
    };
    auto left = [&](int64_t c, int64_t r0, int64_t L, T tau, const T* v) {
        // columns with nonzeros in rows [r0, r0 + L): the band columns up to
        // r0 + L - 1 + b; left of r0 these rows are zero (below the diagonal
        // and outside this step's bulge)
        int64_t w0 = r0, w1 = std::min<int64_t>(n - 1, r0 + L - 1 + b);
        for (int64_t jj = w0; jj <= w1; ++jj) {
            if (jj == c) continue;
            T* __restrict__ col = &a(r0, jj);
            const T s = dotc(L, v, col) * cj(tau);
            if (s != T(0)) for (int64_t t = 0; t < L; ++t) col[t] -= v[t] * s;
        }
    };
    // Sweeps pipelined over threads as in hb2st: step t of sweep j touches
    // rows [c0 - b, c0 + b) x columns [c0, c0 + 2b) with c0 = j + 1 + t b
    // (right update rows [c0 - b, c0 + L) x columns [c0, c0 + L), left update
    // rows [c0, c0 + L) x columns up to c0 + L - 1 + b); sweep j-1's step t'
    // sits at c0 - 1 + (t' - t) b, whose rectangle shares elements with this
    // one only for t' <= t + 2, so step t may run once sweep j-1 has finished
    // its steps 0..t+2 (the chain of lags bounds the whole reduction: lag 3
    // instead of 6 halves it).  Reflectors are kept per sweep and concatenated
    // in sweep order (out-of-order ones commute).
    const int64_t nsw = n > 1 ? n - 1 : 0;
    constexpr int64_t kLag = 3;
    std::vector<Reflectors<T>> QUs(nsw), QVs(nsw);
    struct St { int64_t j, r, c0, c1; };
    const bool par = nsw >= 64 && n >= 8 * b;
    std::vector<std::vector<T>> vs(size_t(par ? omp_get_max_threads() : 1)), ws(vs.size());
    for (auto& x : vs) x.resize(size_t(b + 1));
    for (auto& x : ws) x.resize(size_t(std::max<int64_t>(m, 1)));
    pipelined_sweeps(nsw, kLag, par,
        [&](int64_t j) { return St{j, j, j + 1, std::min(j + b, n - 1)}; },
        [&](St& q, int tid) {
            T* v = vs[tid].data();
            T* w = ws[tid].data();
            const int64_t j = q.j, r = q.r, c0 = q.c0, c1 = q.c1;
            // right reflector: row r, columns [c0, c1]
            const int64_t L = c1 - c0 + 1;
            if (L >= 2) {
                T alpha = cj(a(r, c0));
                for (int64_t t = 1; t < L; ++t) v[t] = cj(a(r, c0 + t));
                T tau;
                larfg(L, alpha, v + 1, 1, tau);
                v[0] = T(1);
                a(r, c0) = cj(alpha);
                for (int64_t t = 1; t < L; ++t) a(r, c0 + t) = T(0);
                if (tau != T(0)) { right(r, c0, L, tau, v, w); QVs[j].push(c0, L, tau, v, j); }
            }
            // left reflector: column c0, rows [c0, min(c1, m-1)]
            const int64_t r1 = std::min(c1, m - 1);
            const int64_t Ll = r1 - c0 + 1;
            if (Ll >= 2) {
                T alpha = a(c0, c0);
                for (int64_t t = 1; t < Ll; ++t) v[t] = a(c0 + t, c0);
                T tau;
                larfg(Ll, alpha, v + 1, 1, tau);
                v[0] = T(1);
                a(c0, c0) = alpha;
                for (int64_t t = 1; t < Ll; ++t) a(c0 + t, c0) = T(0);
                if (tau != T(0)) { left(c0, c0, Ll, tau, v); QUs[j].push(c0, Ll, tau, v, j); }
            }
            // next: row c0 beyond its band, columns [c0 + b, c1 + b]
            const int64_t nc0 = c0 + b, nc1 = std::min(c1 + b, n - 1);
            if (nc0 >= n - 1 || nc1 <= nc0) return false;
            q.r = c0; q.c0 = nc0; q.c1 = nc1;
            return true;
        });
    for (int64_t j = 0; j < nsw; ++j) {
        for (size_t q = 0; q < QVs[j].size(); ++q)
            QV.push(QVs[j].off[q], QVs[j].len[q], QVs[j].tau[q], QVs[j].v.data() + QVs[j].voff[q], j);
        for (size_t q = 0; q < QUs[j].size(); ++q)
            QU.push(QUs[j].off[q], QUs[j].len[q], QUs[j].tau[q], QUs[j].v.data() + QUs[j].voff[q], j);
        QVs[j] = Reflectors<T>();
        QUs[j] = Reflectors<T>();
    }
    d.assign(n, R(0));
    e.assign(std::max<int64_t>(n - 1, 0), R(0));
    pu.assign(n, T(1));
    pv.assign(n, T(1));
    // B' = Du B Dv^H with real nonnegative B: v_0 = 1, u_i from d_i, v_{i+1} from e_i
    for (int64_t i = 0; i < n; ++i) {
        T di = a(i, i);
        R ad = std::abs(di);
        pu[i] = ad > R(0) ? di * pv[i] / T(ad) : pv[i];
        d[i] = ad;
        if (i + 1 < n) {
            T ei = a(i, i + 1);
            R ae = std::abs(ei);
            e[i] = ae;
            // conj(u_i) e_i v_{i+1} = |e_i|  =>  v_{i+1} = u_i |e_i| / e_i
            pv[i + 1] = ae > R(0) ? pu[i] * cj(ei) / T(ae) : pu[i];
        }
    }
}

//------------------------------------------------------------------------------
// Implicit QL (EISPACK tql2 formulation); Z columns are the eigenvectors.
template <typename R, typename T>
int64_t steqr(int64_t n, R* d, R* e_in, T* Z, int64_t ldz, int64_t zrows) {
    if (n <= 0) return 0;
    std::vector<R> e(n, R(0));
    for (int64_t i = 0; i + 1 < n; ++i) e[i] = e_in[i];
    const R eps = std::numeric_limits<R>::epsilon();
    R f = 0, tst1 = 0;
    int64_t unconverged = 0;
    std::vector<Rot<R>> rots;
    for (int64_t l = 0; l < n; ++l) {
        tst1 = std::max(tst1, std::abs(d[l]) + std::abs(e[l]));
        int64_t m = l;
        while (m < n - 1 && std::abs(e[m]) > eps * tst1) ++m;
        if (m > l) {
            int iter = 0;
            do {
                if (++iter > 60) { ++unconverged; break; }
                R g = d[l];
                R p = (d[l + 1] - g) / (R(2) * e[l]);
                R r = std::hypot(p, R(1));
                if (p < 0) r = -r;
                d[l] = e[l] / (p + r);
                d[l + 1] = e[l] * (p + r);
                R dl1 = d[l + 1];
                R h = g - d[l];
                for (int64_t i = l + 2; i < n; ++i) d[i] -= h;
                f += h;
                p = d[m];
                R c = 1, c2 = 1, c3 = 1, el1 = e[l + 1], s = 0, s2 = 0;
                rots.clear();
                for (int64_t i = m - 1; i >= l; --i) {
                    c3 = c2; c2 = c; s2 = s;
                    g = c * e[i];
                    h = c * p;
                    r = fast_hypot(p, e[i]);
                    e[i + 1] = s * r;
                    const R rr = R(1) / r;
                    s = e[i] * rr;
                    c = p * rr;
                    p = c * d[i] - s * g;
                    d[i + 1] = h + s * (c * g + s * d[i]);
                    // Z(:, i+1) = s Z(:,i) + c Z(:,i+1); Z(:,i) = c Z(:,i) - s Z(:,i+1)
                    rots.push_back({i, c, s});
                }
                apply_rots(rots, Z, ldz, zrows);
                p = -s * s2 * c3 * el1 * e[l] / dl1;
                e[l] = s * p;
                d[l] = c * p;
            } while (std::abs(e[l]) > eps * tst1);
        }
        d[l] += f;
        e[l] = 0;
    }
    // sort ascending (selection sort keeps column swaps to n)
    for (int64_t i = 0; i + 1 < n; ++i) {
        int64_t k = i;
        for (int64_t j = i + 1; j < n; ++j) if (d[j] < d[k]) k = j;
        if (k != i) {
            std::swap(d[i], d[k]);
            if (Z) for (int64_t r = 0; r < zrows; ++r) std::swap(Z[r + i * ldz], Z[r + k * ldz]);
        }
    }
    return unconverged;
}

/// steqr with every rotation sent to a sink (distributed Z rows): one
/// sink->sweep per QL sweep, rotations in application order (i DEscending,
/// [x y] <- [c x - s y, s x + c y] on columns (i, i+1)); the final ascending
/// sort as one sink->permute.
template <typename R>
int64_t steqr_core(int64_t n, R* d, R* e_in, RotSink<R>* sink) {
    if (n <= 0) return 0;
    std::vector<R> e(n, R(0));
    for (int64_t i = 0; i + 1 < n; ++i) e[i] = e_in[i];
    const R eps = std::numeric_limits<R>::epsilon();
    R f = 0, tst1 = 0;
    int64_t unconverged = 0;
    std::vector<PlaneRot<R>> rots;
    std::vector<PlaneRot<R>> none;
    for (int64_t l = 0; l < n; ++l) {
        tst1 = std::max(tst1, std::abs(d[l]) + std::abs(e[l]));
        int64_t m = l;
        while (m < n - 1 && std::abs(e[m]) > eps * tst1) ++m;
        if (m > l) {
            int iter = 0;
            do {
                if (++iter > 60) { ++unconverged; break; }
                R g = d[l];
                R p = (d[l + 1] - g) / (R(2) * e[l]);
                R r = std::hypot(p, R(1));
                if (p < 0) r = -r;
                d[l] = e[l] / (p + r);
                d[l + 1] = e[l] * (p + r);
                R dl1 = d[l + 1];
                R h = g - d[l];
                for (int64_t i = l + 2; i < n; ++i) d[i] -= h;
                f += h;
                p = d[m];
                R c = 1, c2 = 1, c3 = 1, el1 = e[l + 1], s = 0, s2 = 0;
                rots.clear();
                for (int64_t i = m - 1; i >= l; --i) {
                    c3 = c2; c2 = c; s2 = s;
                    g = c * e[i];
                    h = c * p;
                    r = std::hypot(p, e[i]);
                    e[i + 1] = s * r;
                    s = e[i] / r;
                    c = p / r;
                    p = c * d[i] - s * g;
                    d[i + 1] = h + s * (c * g + s * d[i]);
                    rots.push_back({i, c, s});
                }
                none.clear();
                if (sink) sink->sweep(rots, none);
                p = -s * s2 * c3 * el1 * e[l] / dl1;
                e[l] = s * p;
                d[l] = c * p;
            } while (std::abs(e[l]) > eps * tst1);
        }
        d[l] += f;
        e[l] = 0;
    }
    std::vector<int64_t> perm(n);
    std::iota(perm.begin(), perm.end(), int64_t(0));
    std::stable_sort(perm.begin(), perm.end(), [&](int64_t a, int64_t b) { return d[a] < d[b]; });
    std::vector<R> ds(n);
    for (int64_t i = 0; i < n; ++i) ds[i] = d[perm[i]];
    std::copy(ds.begin(), ds.end(), d);
    if (sink) sink->permute(perm);
    return unconverged;
}

template <typename R>
int64_t sterf(int64_t n, R* d, R* e) {
    return steqr<R, R>(n, d, e, nullptr, 1, 0);
}

//------------------------------------------------------------------------------
// Divide and conquer (Cuppen; deflation as LAPACK laed2; Gu-Eisenstat vectors
// as laed3), split into the reference's stages (stedc_solve.cc, stedc_merge.cc,
// stedc_z_vector.cc, stedc_sort.cc, stedc_deflate.cc, stedc_secular.cc).

template <typename R>
void stedc_z_vector(int64_t n1, int64_t n, R const* Q, int64_t ldq, R sgn, R* z) {
    const R s2 = std::sqrt(R(2));
    for (int64_t j = 0; j < n1; ++j) z[j] = Q[(n1 - 1) + j * ldq] / s2;
    for (int64_t j = n1; j < n; ++j) z[j] = sgn * Q[n1 + j * ldq] / s2;
}

template <typename R>
void stedc_sort(int64_t n, R* D, R* z, R const* Q, int64_t ldq, R* Qp, int64_t ldqp, int64_t* perm) {
    std::iota(perm, perm + n, int64_t(0));
    std::stable_sort(perm, perm + n, [&](int64_t a, int64_t b) { return D[a] < D[b]; });
    std::vector<R> Ds(n), zs(n);
    for (int64_t j = 0; j < n; ++j) {
        Ds[j] = D[perm[j]];
        zs[j] = z[perm[j]];
        std::copy(Q + perm[j] * ldq, Q + perm[j] * ldq + n, Qp + j * ldqp);
    }
    std::copy(Ds.begin(), Ds.end(), D);
    std::copy(zs.begin(), zs.end(), z);
}

template <typename R>
int64_t stedc_deflate(int64_t n, R rho, R* D, R* z, R* Qp, int64_t ldqp, char* deflated) {
    const R eps = std::numeric_limits<R>::epsilon();
    R dmax = 0, zmax = 0;
    for (int64_t j = 0; j < n; ++j) { dmax = std::max(dmax, std::abs(D[j])); zmax = std::max(zmax, std::abs(z[j])); }
    const R tol = R(8) * eps * std::max(dmax, zmax * rho);
    // tiny components of z
    for (int64_t j = 0; j < n; ++j) deflated[j] = (rho * std::abs(z[j]) <= tol) ? 1 : 0;
    // close pairs of D: a Givens rotation of the two Q columns moves all of
    // z onto one of them
    int64_t last = -1;
    for (int64_t j = 0; j < n; ++j) {
        if (deflated[j]) continue;
        if (last >= 0) {
            R t = std::hypot(z[last], z[j]);
            R c = z[j] / t, sn = -z[last] / t;
            if (std::abs((D[j] - D[last]) * c * sn) <= tol) {
                R* ql = Qp + last * ldqp;
                R* qj = Qp + j * ldqp;
                for (int64_t i = 0; i < n; ++i) {
                    R x = ql[i], y = qj[i];
                    ql[i] = c * x + sn * y;
                    qj[i] = -sn * x + c * y;
                }
                R dl = D[last], dj = D[j];
                D[last] = dl * c * c + dj * sn * sn;
                D[j] = dl * sn * sn + dj * c * c;
                z[j] = t;
                z[last] = 0;
                deflated[last] = 1;
            }
        }
        last = j;
    }
    int64_t k = 0;
    for (int64_t j = 0; j < n; ++j) k += !deflated[j];
    return k;
}

template <typename R>
void stedc_secular(int64_t k, R rho, R const* dd, R const* zz, R* lam, R* U, int64_t ldu) {
    if (k <= 0) return;
    R znorm2 = 0;
    for (int64_t i = 0; i < k; ++i) znorm2 += zz[i] * zz[i];
    // roots: lambda_j = dd[org[j]] + tau[j], tau relative to the closer pole
    std::vector<int64_t> org(k);
    std::vector<R> tau(k);
    #pragma omp parallel for schedule(dynamic, 8) if (k > 64)
    for (int64_t j = 0; j < k; ++j) {
        int64_t o2 = j;
        tau[j] = secular::root<R>(k, j, rho, dd, zz, znorm2, &o2);
        org[j] = o2;
    }
    // Gu-Eisenstat: recompute z from the computed roots
    auto lam_minus_d = [&](int64_t j, int64_t i) { return (dd[org[j]] - dd[i]) + tau[j]; };
    std::vector<R> zh(k);
    for (int64_t i = 0; i < k; ++i) {
        R pr = lam_minus_d(k - 1, i) / rho;
        for (int64_t j = 0; j < k - 1; ++j) {
            R num = lam_minus_d(j, i);
            R den = (j < i) ? (dd[j] - dd[i]) : (dd[j + 1] - dd[i]);
            pr *= num / den;
        }
        zh[i] = std::copysign(std::sqrt(std::abs(pr)), zz[i]);
    }
    // eigenvectors of D + rho z z^T
    #pragma omp parallel for schedule(static) if (k > 256)
    for (int64_t j = 0; j < k; ++j) {
        R nrm = 0;
        for (int64_t i = 0; i < k; ++i) {
            R u = zh[i] / ((dd[i] - dd[org[j]]) - tau[j]);
            U[i + j * ldu] = u;
            nrm += u * u;
        }
        nrm = std::sqrt(nrm);
        for (int64_t i = 0; i < k; ++i) U[i + j * ldu] /= nrm;
        lam[j] = dd[org[j]] + tau[j];
    }
}

namespace {
/// Merge-product hook: C = A * B on the GPU when one is attached (set by the
/// device layer); the host blocked gemm otherwise.
StedcGemm g_stedc_gemm = nullptr;
}

void set_stedc_gemm(StedcGemm f) { g_stedc_gemm = f; }

template <typename R>
void stedc_solve(int64_t n, R* d, R* e, R* Q, int64_t ldq) {
    const int64_t SMALL = 32;
    if (n <= SMALL) {
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < n; ++i) Q[i + j * ldq] = (i == j) ? R(1) : R(0);
        steqr<R, R>(n, d, e, Q, ldq, n);
        return;
    }
    // divide: T = diag(T1, T2) + |beta| v v^T with the coupling removed
    const int64_t m = n / 2;
    const R beta = e[m - 1];
    const R rho0 = std::abs(beta);
    d[m - 1] -= rho0;
    d[m] -= rho0;
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < n; ++i) Q[i + j * ldq] = R(0);
    stedc_solve(m, d, e, Q, ldq);
    stedc_solve(n - m, d + m, e + m, Q + m + m * ldq, ldq);
    // conquer
    std::vector<R> z(n), Qp(size_t(n) * n);
    std::vector<int64_t> perm(n);
    stedc_z_vector<R>(m, n, Q, ldq, beta < 0 ? R(-1) : R(1), z.data());
    const R rho = R(2) * rho0;
    stedc_sort<R>(n, d, z.data(), Q, ldq, Qp.data(), n, perm.data());
    std::vector<char> defl(n);
    const int64_t k = stedc_deflate<R>(n, rho, d, z.data(), Qp.data(), n, defl.data());
    std::vector<R> lam(n), Qout(size_t(n) * n, R(0));
    if (k > 0) {
        std::vector<int64_t> act;
        for (int64_t j = 0; j < n; ++j) if (!defl[j]) act.push_back(j);
        // the rotations may leave the active D out of order
        std::sort(act.begin(), act.end(), [&](int64_t a, int64_t b) { return d[a] < d[b]; });
        std::vector<R> dd(k), zz(k), U(size_t(k) * k), Qa(size_t(n) * k);
        for (int64_t i = 0; i < k; ++i) {
            dd[i] = d[act[i]];
            zz[i] = z[act[i]];
            std::copy(Qp.begin() + act[i] * n, Qp.begin() + act[i] * n + n, Qa.begin() + i * n);
        }
        stedc_secular<R>(k, rho, dd.data(), zz.data(), lam.data(), U.data(), k);
        // merge product: Qout(:, 0:k) = Qa * U
        if (g_stedc_gemm && n * k >= 512 * 512)
            g_stedc_gemm(sizeof(R), n, k, k, Qa.data(), n, U.data(), k, Qout.data(), n);
        else
            gemm<R>(Op::NoTrans, Op::NoTrans, n, k, k, R(1), Qa.data(), n, U.data(), k, R(0), Qout.data(), n);
    }
    // deflated columns pass through
    int64_t col = k;
    for (int64_t j = 0; j < n; ++j) {
        if (!defl[j]) continue;
        lam[col] = d[j];
        std::copy(Qp.begin() + j * n, Qp.begin() + j * n + n, Qout.begin() + col * n);
        ++col;
    }
    // sort ascending into d, Q
    std::vector<int64_t> o(n);
    std::iota(o.begin(), o.end(), int64_t(0));
    std::sort(o.begin(), o.end(), [&](int64_t a, int64_t b) { return lam[a] < lam[b]; });
    for (int64_t j = 0; j < n; ++j) {
        d[j] = lam[o[j]];
        std::copy(Qout.begin() + o[j] * n, Qout.begin() + o[j] * n + n, Q + j * ldq);
    }
}

template <typename R>
int64_t stedc(int64_t n, R* d, R* e, R* Q, int64_t ldq) {
    if (n <= 0) return 0;
    std::vector<R> ee(e, e + std::max<int64_t>(n - 1, 0));
    ee.push_back(R(0));
    stedc_solve<R>(n, d, ee.data(), Q, ldq);
    return 0;
}

//------------------------------------------------------------------------------
// Golub-Reinsch implicit-shift QR on the upper bidiagonal (EISPACK svd).
template <typename R>
int64_t bdsqr_core(int64_t n, R* w, R* e, RotSink<R>* sink) {
    if (n <= 0) return 0;
    std::vector<R> rv1(n, R(0));
    for (int64_t i = 1; i < n; ++i) rv1[i] = e[i - 1];
    R anorm = 0;
    for (int64_t i = 0; i < n; ++i) anorm = std::max(anorm, std::abs(w[i]) + std::abs(rv1[i]));
    int64_t fail = 0;
    // Rot convention of the sink: [x y] <- [c x - s y, s x + c y]; the sweep
    // below rotates [x y] <- [c x + s y, c y - s x], i.e. (c, -s).
    std::vector<PlaneRot<R>> ru, rv;
    for (int64_t k = n - 1; k >= 0; --k) {
        for (int its = 0; its < 75; ++its) {
            bool flag = true;
            int64_t l = k, nm = 0;
            for (; l >= 0; --l) {
                nm = l - 1;
                if (l == 0 || std::abs(rv1[l]) + anorm == anorm) { flag = false; break; }
                if (std::abs(w[nm]) + anorm == anorm) break;
            }
            if (flag) {
                R c = 0, s = 1;
                for (int64_t i = l; i <= k; ++i) {
                    R f = s * rv1[i];
                    rv1[i] = c * rv1[i];
                    if (std::abs(f) + anorm == anorm) break;
                    R g = w[i];
                    R h = std::hypot(f, g);
                    w[i] = h;
                    h = R(1) / h;
                    c = g * h;
                    s = -f * h;
                    if (sink) sink->rot_u(nm, i, c, s);
                }
            }
            R z = w[k];
            if (l == k) {
                if (z < R(0)) {
                    w[k] = -z;
                    if (sink) sink->negate_v(k);
                }
                break;
            }
            if (its == 74) { ++fail; break; }
            R x = w[l];
            nm = k - 1;
            R y = w[nm], g = rv1[nm], h = rv1[k];
            R f = ((y - z) * (y + z) + (g - h) * (g + h)) / (R(2) * h * y);
            g = std::hypot(f, R(1));
            f = ((x - z) * (x + z) + h * ((y / (f + std::copysign(g, f))) - h)) / x;
            R c = 1, s = 1;
            ru.clear(); rv.clear();
            ru.reserve(size_t(nm - l + 1)); rv.reserve(size_t(nm - l + 1));
            for (int64_t j = l; j <= nm; ++j) {
                int64_t i = j + 1;
                g = rv1[i];
                y = w[i];
                h = s * g;
                g = c * g;
                z = fast_hypot(f, h);
                rv1[j] = z;
                const R rz = R(1) / z;
                c = f * rz;
                s = h * rz;
                f = x * c + g * s;
                g = g * c - x * s;
                h = y * s;
                y *= c;
                rv.push_back(PlaneRot<R>{j, c, -s});
                z = fast_hypot(f, h);
                w[j] = z;
                if (z != R(0)) {
                    z = R(1) / z;
                    c = f * z;
                    s = h * z;
                }
                f = c * g + s * y;
                x = c * y - s * g;
                ru.push_back(PlaneRot<R>{j, c, -s});
            }
            if (sink) sink->sweep(ru, rv);
            rv1[l] = 0;
            rv1[k] = f;
            w[k] = x;
        }
    }
    // sort descending (selection sort: the permutation goes to the sink)
    std::vector<int64_t> perm(n);
    for (int64_t i = 0; i < n; ++i) perm[i] = i;
    bool moved = false;
    for (int64_t i = 0; i + 1 < n; ++i) {
        int64_t kk = i;
        for (int64_t j = i + 1; j < n; ++j) if (w[j] > w[kk]) kk = j;
        if (kk != i) { std::swap(w[i], w[kk]); std::swap(perm[i], perm[kk]); moved = true; }
    }
    if (sink && moved) sink->permute(perm);
    return fail;
}

namespace {

/// host backend: U and Vt = VT^T in host memory (row blocks of the
/// rotations in parallel, apply_rots)
template <typename R, typename T>
struct HostRotSink : RotSink<R> {
    T* U; int64_t ldu, urows;
    T* V; int64_t vcols;
    std::vector<Rot<R>> tu, tv;
    void sweep(std::vector<PlaneRot<R>>& ru, std::vector<PlaneRot<R>>& rv) override {
        tv.clear(); tu.clear();
        for (auto const& r : rv) tv.push_back(Rot<R>{r.i, r.c, r.s});
        for (auto const& r : ru) tu.push_back(Rot<R>{r.i, r.c, r.s});
        apply_rots(tv, V, vcols, vcols);
        apply_rots(tu, U, ldu, urows);
    }
    void rot_u(int64_t a, int64_t b, R c, R s) override {
        if (!U) return;
        T* x = U + a * ldu;
        T* y = U + b * ldu;
        for (int64_t r = 0; r < urows; ++r) {
            T ya = x[r], yb = y[r];
            x[r] = ya * c + yb * s;
            y[r] = yb * c - ya * s;
        }
    }
    void negate_v(int64_t k) override {
        if (V) for (int64_t jj = 0; jj < vcols; ++jj) V[jj + k * vcols] = -V[jj + k * vcols];
    }
    void permute(std::vector<int64_t> const& perm) override {
        const int64_t n = int64_t(perm.size());
        auto perm_cols = [&](T* M, int64_t ld, int64_t rows) {
            if (!M) return;
            std::vector<T> tmp(size_t(rows) * n);
            for (int64_t i = 0; i < n; ++i)
                for (int64_t r = 0; r < rows; ++r) tmp[r + i * rows] = M[r + perm[i] * ld];
            for (int64_t i = 0; i < n; ++i)
                for (int64_t r = 0; r < rows; ++r) M[r + i * ld] = tmp[r + i * rows];
        };
        perm_cols(U, ldu, urows);
        perm_cols(V, vcols, vcols);
    }
};

}  // namespace

template <typename R, typename T>
int64_t bdsqr(int64_t n, R* w, R* e, T* U, int64_t ldu, int64_t urows, T* VT, int64_t ldvt, int64_t vcols) {
    if (n <= 0) return 0;
    // VT is rotated by rows; rows of a column-major VT are ld-strided, so work
    // on Vt = VT^T (row j of VT = contiguous column j of Vt) and transpose back
    std::vector<T> Vt;
    if (VT) {
        Vt.resize(size_t(vcols) * n);
        for (int64_t jj = 0; jj < vcols; ++jj)
            for (int64_t j = 0; j < n; ++j) Vt[jj + j * vcols] = VT[j + jj * ldvt];
    }
    HostRotSink<R, T> sink;
    sink.U = U; sink.ldu = ldu; sink.urows = urows;
    sink.V = VT ? Vt.data() : nullptr; sink.vcols = vcols;
    int64_t fail = bdsqr_core<R>(n, w, e, (U || VT) ? &sink : nullptr);
    if (VT) {
        for (int64_t jj = 0; jj < vcols; ++jj)
            for (int64_t j = 0; j < n; ++j) VT[j + jj * ldvt] = Vt[jj + j * vcols];
    }
    return fail;
}

//------------------------------------------------------------------------------
#define SLATE_EIGH_INST(T)                                                                              \
    template struct Reflectors<T>;                                                                      \
    template void hb2st<T>(int64_t, int64_t, T*, int64_t, std::vector<real_type<T>>&,                   \
                           std::vector<real_type<T>>&, Reflectors<T>&, std::vector<T>&);                \
    template void tb2bd<T>(int64_t, int64_t, int64_t, T*, int64_t, std::vector<real_type<T>>&,          \
                           std::vector<real_type<T>>&, Reflectors<T>&, Reflectors<T>&, std::vector<T>&, \
                           std::vector<T>&);                                                            \
    template int64_t steqr<real_type<T>, T>(int64_t, real_type<T>*, real_type<T>*, T*, int64_t, int64_t); \
    template int64_t bdsqr<real_type<T>, T>(int64_t, real_type<T>*, real_type<T>*, T*, int64_t, int64_t, \
                                            T*, int64_t, int64_t);

SLATE_EIGH_INST(float)
SLATE_EIGH_INST(double)
SLATE_EIGH_INST(std::complex<float>)
SLATE_EIGH_INST(std::complex<double>)

template int64_t bdsqr_core<float>(int64_t, float*, float*, RotSink<float>*);
template int64_t bdsqr_core<double>(int64_t, double*, double*, RotSink<double>*);
template int64_t sterf<float>(int64_t, float*, float*);
template int64_t steqr_core<float>(int64_t, float*, float*, RotSink<float>*);
template int64_t steqr_core<double>(int64_t, double*, double*, RotSink<double>*);
template int64_t sterf<double>(int64_t, double*, double*);
template int64_t stedc<float>(int64_t, float*, float*, float*, int64_t);
template int64_t stedc<double>(int64_t, double*, double*, double*, int64_t);
#define SLATE_STEDC_INST(R)                                                                           \
    template void stedc_z_vector<R>(int64_t, int64_t, R const*, int64_t, R, R*);                      \
    template void stedc_sort<R>(int64_t, R*, R*, R const*, int64_t, R*, int64_t, int64_t*);            \
    template int64_t stedc_deflate<R>(int64_t, R, R*, R*, R*, int64_t, char*);                       \
    template void stedc_secular<R>(int64_t, R, R const*, R const*, R*, R*, int64_t);                  \
    template void stedc_solve<R>(int64_t, R*, R*, R*, int64_t);
SLATE_STEDC_INST(float)
SLATE_STEDC_INST(double)

}  // namespace host
}  // namespace slate
