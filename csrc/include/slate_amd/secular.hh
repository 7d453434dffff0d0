// Secular-equation root finder shared by the host divide-and-conquer
// (eig_host.cc stedc_secular, eig_dist.cc secular_host) and the device
// kernel (kernels/stedc.hip secular_roots_kernel): one definition, compiled
// by g++ for the host and by hipcc for gfx950 (reference src/stedc_secular.cc
// calls LAPACK laed4 per root; this is the same rational "middle way"
// iteration, written from its derivation below, with a bisection safeguard).
//
// Root j of  w(lambda) = 1/rho + sum_i z_i^2 / (d_i - lambda),  d ascending,
// rho > 0, lies in (d_j, d_{j+1}) (d_k := d_{k-1} + rho |z|^2 for the last).
// It is returned as tau = lambda - d_o relative to the NEARER pole o (j or
// j + 1): the Gu-Eisenstat vectors need lambda - d_i to full relative
// precision, which the difference of two absolute values would lose.
//
// Iteration at t (shifted coordinates, delta_i = (d_i - d_o) - t): split w
// into psi (poles i <= j, left of the root) and phi (i > j), model
//   w(t + eta) ~ c + s / (delta_j - eta) + S / (delta_{j+1} - eta)
// with s = delta_j^2 psi', S = delta_{j+1}^2 phi' (derivatives matched per
// side) and c = w - delta_j psi' - delta_{j+1} phi' (value matched), and take
// the root of  c eta^2 - A eta + B = 0,
//   A = (delta_j + delta_{j+1}) w - delta_j delta_{j+1} (psi' + phi'),
//   B = delta_j delta_{j+1} w,
// in its cancellation-free form.  The model is exact for a two-pole w, so
// the step converges in a handful of iterations where the previous pure
// bisection needed 60-400 evaluations of the O(k) sum per root (the device
// merge's secular stage was 465 of 488 ms of stedc at n = 8192).  A step
// that leaves the sign bracket [a, b] falls back to bisection; the loop
// stops when |w| is at its rounding level, eps (8 (|psi| + |phi|) + 1/rho +
// |t| (psi' + phi')).
#pragma once

#include <cmath>
#include <cstdint>
#include <limits>

#if defined(__HIPCC__)
#define SLATE_SECULAR_FN __host__ __device__ inline
#else
#define SLATE_SECULAR_FN inline
#endif

namespace slate {
namespace secular {

template <typename R>
struct Sums {
    R psi = 0, phi = 0, dpsi = 0, dphi = 0;
};

/// psi / phi and their derivatives at shifted point t (origin pole o).
template <typename R>
SLATE_SECULAR_FN Sums<R> sums(int64_t k, int64_t j, const R* d, const R* z, int64_t o, R t) {
    Sums<R> s;
    const R d0 = d[o];
    for (int64_t i = 0; i <= j; ++i) {
        const R r = z[i] / ((d[i] - d0) - t);
        s.psi += z[i] * r;
        s.dpsi += r * r;
    }
    for (int64_t i = j + 1; i < k; ++i) {
        const R r = z[i] / ((d[i] - d0) - t);
        s.phi += z[i] * r;
        s.dphi += r * r;
    }
    return s;
}

/// Root j (0-based) of the secular equation; *org receives the origin pole.
/// sum_fn(o, t) -> Sums<R> evaluates psi / phi and their derivatives (the
/// serial `sums` here; the device kernel passes a wave-parallel one, every
/// lane then runs the same iteration on the same reduced values).
template <typename R, typename SumFn>
SLATE_SECULAR_FN R root_with(int64_t k, int64_t j, R rho, const R* d, R znorm2, int64_t* org, SumFn&& sum_fn) {
    const R eps = std::numeric_limits<R>::epsilon();
    const R rhoinv = R(1) / rho;
    const bool last = j + 1 >= k;
    const R gap = last ? rho * znorm2 : d[j + 1] - d[j];
    int64_t o = j;
    R a = 0, b = gap, t = gap / 2;
    if (!last) {
        // the sign of w at the midpoint picks the half, and with it the
        // nearer pole as origin
        const Sums<R> s = sum_fn(j, gap / 2);
        if (rhoinv + s.psi + s.phi < R(0)) { o = j + 1; a = -gap / 2; b = 0; t = -gap / 4; }
        else { b = gap / 2; t = gap / 4; }
    }
    const R dj0 = d[j] - d[o], dj1 = last ? R(0) : d[j + 1] - d[o];
    for (int it = 0; it < 200; ++it) {
        const Sums<R> s = sum_fn(o, t);
        const R w = rhoinv + s.psi + s.phi;
        if (w == R(0)) break;
        if (w > R(0)) b = t; else a = t;
        const R dw = s.dpsi + s.dphi;
        const R erretm = R(8) * (s.phi - s.psi) + rhoinv + std::fabs(t) * dw;
        if (std::fabs(w) <= eps * erretm) break;
        const R Dj = dj0 - t;
        R eta;
        if (!last) {
            const R Dj1 = dj1 - t;
            const R C = w - Dj * s.dpsi - Dj1 * s.dphi;
            const R A = (Dj + Dj1) * w - Dj * Dj1 * dw;
            const R B = Dj * Dj1 * w;
            const R disc = std::sqrt(std::fabs(A * A - R(4) * B * C));
            if (C == R(0)) eta = B / A;
            else if (A <= R(0)) eta = (A - disc) / (R(2) * C);
            else eta = R(2) * B / (A + disc);
        } else {
            const R C = w - Dj * s.dpsi;
            eta = Dj + Dj * Dj * s.dpsi / C;
        }
        // the step must point toward the root (w increases with t)
        if (!(w * eta < R(0))) eta = -w / dw;
        R tn = t + eta;
        if (!(tn > a && tn < b)) tn = (a + b) / 2;
        if (tn == t) break;
        t = tn;
        if (b - a <= R(2) * eps * std::fmax(std::fabs(a), std::fabs(b))) break;
    }
    *org = o;
    return t;
}

template <typename R>
SLATE_SECULAR_FN R root(int64_t k, int64_t j, R rho, const R* d, const R* z, R znorm2, int64_t* org) {
    return root_with<R>(k, j, rho, d, znorm2, org, [&](int64_t o, R t) { return sums(k, j, d, z, o, t); });
}

}  // namespace secular
}  // namespace slate

#undef SLATE_SECULAR_FN
