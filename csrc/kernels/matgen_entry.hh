// Element formulas of the test-matrix generator, shared by the device kernel
// (kernels/matgen.hip) and the host path (src/matgen.cc) so both targets and
// every process grid produce bit-identical matrices.  Kinds follow the
// reference's generate_matrix list (matgen/generate_matrix_ge.cc:84-283,
// generate_matrix_utils.cc:64-125); the random source is a counter hash of
// (global i, global j, seed) in place of the reference's Philox-2x64
// (matgen/random.cc:53-110) -- same property: values do not depend on the
// distribution of the matrix.
#pragma once

#include <cmath>
#include <cstdint>

#ifndef SLATE_HD
#if defined(__HIPCC__) || defined(__HIP__)
#define SLATE_HD __host__ __device__
#else
#define SLATE_HD
#endif
#endif

namespace slate_amd {
namespace gen {

enum Code : int {
    Zeros, Ones, Identity, Ij, Jordan, JordanT, Chebspec, Circul, Fiedler, Gfpp, Kms, Orthog,
    Riemann, Ris, ZielkeNS,
    Rand, Rands, Randn, Randb, Randr,  // random kinds (shift / scale apply)
    Diag,                              // A = diag(sigma), sigma from a vector
    SymRands,                          // Hermitian rands (+ shift on diagonal): fast SPD for benchmarks
};

/// Everything a thread needs to compute element (i, j) of the view.
struct Spec {
    int code;
    uint64_t seed;
    int64_t m, n, max_mn;
    double ij_scale;     // ij: 10^-ceil(log10(n))
    double shift;        // added to the diagonal (dominant / spd)
    double scale;        // sigma_max (random kinds)
    const double* sigma; // Diag: sigma[i] (device or host pointer matching the target)
};

SLATE_HD inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27; x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

/// uniform [0, 1) from the (i, j, seed) counter
SLATE_HD inline double unit(uint64_t i, uint64_t j, uint64_t seed) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull ^ (j + 0x632BE59BD9B4E019ull) * 0xD1B54A32D192ED03ull
               ^ seed * 0x94D049BB133111EBull;
    return double(mix64(x) >> 11) * (1.0 / 9007199254740992.0);
}

/// one sample of the random kind `code`; `stream` separates real / imaginary parts
SLATE_HD inline double rand_sample(int code, uint64_t i, uint64_t j, uint64_t seed) {
    double u = unit(i, j, seed);
    switch (code) {
        case Rand: return u;
        case Randb: return u < 0.5 ? 0.0 : 1.0;
        case Randr: return u < 0.5 ? -1.0 : 1.0;
        case Randn: {
            // Box-Muller on two independent counters; 1 - u in (0, 1] avoids log(0)
            double v = unit(i, j, seed ^ 0x5851F42D4C957F2Dull);
            return sqrt(-2.0 * log(1.0 - u)) * cos(6.283185307179586 * v);
        }
        default: return 2.0 * u - 1.0;  // Rands, SymRands
    }
}

/// Real part (re) and imaginary part (im) of element (i, j); `cplx` selects
/// whether random kinds draw an imaginary part.
SLATE_HD inline void entry(Spec const& s, int64_t i, int64_t j, bool cplx, double& re, double& im) {
    const double pi = 3.14159265358979323846;
    im = 0.0;
    switch (s.code) {
        case Zeros: re = 0.0; return;
        case Ones: re = 1.0; return;
        case Identity: re = i == j ? 1.0 : 0.0; return;
        case Ij: re = double(i) + double(j) * s.ij_scale; return;
        case Jordan: re = (i == j || i + 1 == j) ? 1.0 : 0.0; return;
        case JordanT: re = (i == j || i == j + 1) ? 1.0 : 0.0; return;
        case Chebspec: {
            const int64_t N = s.max_mn;
            double xi = cos(pi * double(i + 1) / double(N));
            double xj = cos(pi * double(j + 1) / double(N));
            if (i != j) {
                double ci = i == N - 1 ? 2.0 : 1.0, cj = j == N - 1 ? 2.0 : 1.0;
                double sg = ((i + j) % 2 == 0) ? 1.0 : -1.0;
                re = sg * ci / (cj * (xj - xi));
            } else if (j + 1 == N) {
                re = -(2.0 * double(N) * double(N) + 1.0) / 6.0;
            } else {
                re = -0.5 * xi / (1.0 - xi * xi);
            }
            return;
        }
        case Circul: { int64_t d = j - i; re = double(d + (d < 0 ? s.max_mn : 0) + 1); return; }
        case Fiedler: re = double(i > j ? i - j : j - i); return;
        case Gfpp: re = j == s.n - 1 ? 1.0 : (i > j ? -1.0 : (i == j ? 0.5 : 0.0)); return;
        case Kms: re = pow(0.5, double(i > j ? i - j : j - i)); return;
        case Orthog: {
            double N1 = double(s.max_mn + 1);
            re = sqrt(2.0 / N1) * sin(double(i) * double(j) * pi / N1);
            return;
        }
        case Riemann: re = ((j + 2) % (i + 2) == 0) ? double(j + 1) : -1.0; return;
        case Ris: re = 0.5 / (double(s.max_mn - j - i) + 1.5); return;
        case ZielkeNS: re = j < i ? 1.0 : ((j + 1 == s.max_mn && i == 0) ? -1.0 : 0.0); return;
        case Diag: re = (i == j && s.sigma) ? s.sigma[i] : 0.0; return;
        case SymRands: {
            uint64_t a = uint64_t(i < j ? i : j), b = uint64_t(i < j ? j : i);
            re = rand_sample(Rands, a, b, s.seed);
            if (cplx) {
                double w = rand_sample(Rands, a, b, s.seed + 7919);
                im = i == j ? 0.0 : (i < j ? -w : w);
            }
            if (i == j) re += s.shift;
            re *= s.scale; im *= s.scale;
            return;
        }
        default: {  // Rand, Rands, Randn, Randb, Randr
            re = rand_sample(s.code, uint64_t(i), uint64_t(j), s.seed);
            if (cplx) im = rand_sample(s.code, uint64_t(i), uint64_t(j), s.seed + 7919);
            if (i == j) re += s.shift;
            re *= s.scale; im *= s.scale;
            return;
        }
    }
}

}  // namespace gen
}  // namespace slate_amd
