// Test-matrix generator (reference matgen/: generate_matrix(MatgenParams, A)).
#pragma once

#include "matrix.hh"

#include <string>

namespace slate {

/// Fill A with a grid-independent test matrix.  kind: "rands" (uniform
/// [-1,1)), "rand" ([0,1)), "spd" (Hermitian rands + shift*I, shift<0 -> n),
/// "diag_dominant" (rands + shift*I), "identity", "zeros".
template <typename T>
void generate_matrix(std::string const& kind, BaseMatrix<T>& A, uint64_t seed = 42, double shift = -1,
                     Options const& opts = {});

}  // namespace slate
