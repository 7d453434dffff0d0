// Small utilities (reference include/slate/internal/util.hh:27-290).
#pragma once

#include "types.hh"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <map>
#include <string>

namespace slate {

inline int64_t ceildiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t roundup(int64_t a, int64_t b) { return ceildiv(a, b) * b; }

/// NaN-propagating max (util.hh max_nan)
template <typename R>
inline R max_nan(R x, R y) { return (std::isnan(y) || y >= x) ? y : x; }

/// Combine two (scale, sumsq) pairs as in LAPACK lassq (util.hh combine_sumsq).
template <typename R>
inline void combine_sumsq(R& scale1, R& sumsq1, R scale2, R sumsq2) {
    if (scale1 > scale2) {
        if (scale1 != 0) sumsq1 = sumsq1 + sumsq2 * (scale2 / scale1) * (scale2 / scale1);
    } else if (scale2 != 0) {
        sumsq1 = sumsq1 * (scale1 / scale2) * (scale1 / scale2) + sumsq2;
        scale1 = scale2;
    }
}

/// Accumulate |x| into (scale, sumsq).
template <typename R>
inline void add_sumsq(R& scale, R& sumsq, R absx) {
    if (absx != 0) {
        if (scale < absx) { sumsq = 1 + sumsq * (scale / absx) * (scale / absx); scale = absx; }
        else sumsq += (absx / scale) * (absx / scale);
    }
}

//------------------------------------------------------------------------------
// Block-cyclic index maps (ScaLAPACK numroc / indxl2g / indxg2l semantics,
// reference util.hh local2global/global2local/num_local_rows_cols :179-265).

/// Number of indices in [0, n) owned by process `iproc` of `nprocs` with block
/// size nb (first block on process 0).
inline int64_t numroc(int64_t n, int64_t nb, int iproc, int nprocs) {
    int64_t nblocks = n / nb;
    int64_t num = (nblocks / nprocs) * nb;
    int64_t extra = nblocks % nprocs;
    if (iproc < extra) num += nb;
    else if (iproc == extra) num += n % nb;
    return num;
}

/// Number of indices in [0, g) owned by iproc: local index of the first owned
/// global index >= g (i.e., a "ceil" global->local map).
inline int64_t g2l_ceil(int64_t g, int64_t nb, int iproc, int nprocs) {
    return numroc(g, nb, iproc, nprocs);
}

/// Global index of local index l on process iproc.
inline int64_t l2g(int64_t l, int64_t nb, int iproc, int nprocs) {
    return ((l / nb) * nprocs + iproc) * nb + l % nb;
}

/// Local index of global index g (which must be owned by its process).
inline int64_t g2l(int64_t g, int64_t nb, int nprocs) {
    return (g / (nb * nprocs)) * nb + g % nb;
}

inline int owner(int64_t g, int64_t nb, int nprocs) { return int((g / nb) % nprocs); }

//------------------------------------------------------------------------------
/// Wall-clock timer (reference util.hh Timer :267-290).
class Timer {
public:
    Timer() { reset(); }
    void reset() { t0_ = std::chrono::steady_clock::now(); }
    double elapsed() const {
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0_).count();
    }
private:
    std::chrono::steady_clock::time_point t0_;
};

/// Global timers map filled by drivers (reference src/core/types.cc:23).
std::map<std::string, double>& timers();

/// Library version string (reference src/version.cc).
const char* version();
const char* id();

}  // namespace slate
