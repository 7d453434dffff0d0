// Test-matrix generator (reference include/slate/generate_matrix.hh,
// matgen/generate_matrix_*.cc).
#pragma once

#include "matrix.hh"

#include <cmath>
#include <limits>
#include <string>
#include <vector>

namespace slate {

/// Parameters of generate_matrix (reference MatgenParams).
/// kind = base[_distribution][_scaling][_modifier...]; see generate_matrix_usage().
struct MatgenParams {
    std::string kind = "rands";
    double cond_request = std::numeric_limits<double>::quiet_NaN();  ///< NaN: 1/sqrt(eps)
    double condD = std::numeric_limits<double>::quiet_NaN();         ///< NaN: 1 (no D scaling)
    int64_t seed = 42;
    double cond_actual = std::numeric_limits<double>::quiet_NaN();   ///< output: cond of the result, NaN if unknown
    int verbose = 0;
};

/// Help text listing the kinds, distributions, scalings and modifiers.
std::string generate_matrix_usage();

/// General m x n test matrix; Sigma receives singular values / eigenvalues when
/// known (NaN otherwise).  Kinds: zeros ones identity ij jordan jordanT chebspec
/// circul fiedler gfpp kms orthog riemann ris zielkeNS rand rands randn randb
/// randr diag svd poev|spd heev|syev geev.
template <typename T>
void generate_matrix(MatgenParams& params, Matrix<T>& A, std::vector<real_type<T>>& Sigma,
                     Options const& opts = {});
template <typename T>
void generate_matrix(MatgenParams& params, Matrix<T>& A, Options const& opts = {});

/// Trapezoid / triangular / symmetric / Hermitian test matrix (the stored
/// triangle is generated; Hermitian diagonals are made real).
template <typename T>
void generate_matrix(MatgenParams& params, BaseTrapezoidMatrix<T>& A, std::vector<real_type<T>>& Sigma,
                     Options const& opts = {});

/// Fast grid-independent fill used by benchmarks and tests: any element kind
/// above, plus "spd" (Hermitian rands + shift*I, shift < 0 -> max(m, n)) and
/// "diag_dominant" / "rands+n" (rands + shift*I).
template <typename T>
void generate_matrix(std::string const& kind, BaseMatrix<T>& A, uint64_t seed = 42, double shift = -1,
                     Options const& opts = {});

}  // namespace slate
