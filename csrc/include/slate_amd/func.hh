// Distribution functions (reference include/slate/func.hh:39-339): lambdas
// describing tile sizes, tile->rank and tile->device maps.  Storage in this
// framework is always 2D block-cyclic over a Grid; these functions describe
// (and are checked against) that layout and are provided for API parity.
#pragma once

#include "enums.hh"

#include <cstdint>
#include <functional>
#include <tuple>

namespace slate {
namespace func {

using ij_tuple = std::tuple<int64_t, int64_t>;

/// uniform block size: tile i has nb rows except the last (func.hh:39)
inline std::function<int64_t(int64_t)> uniform_blocksize(int64_t n, int64_t nb) {
    return [n, nb](int64_t i) { return (i + 1) * nb > n ? n - i * nb : nb; };
}

/// 2D block-cyclic process map (func.hh:179)
inline std::function<int(ij_tuple)> process_2d_grid(GridOrder order, int p, int q) {
    return [order, p, q](ij_tuple ij) {
        int64_t i = std::get<0>(ij), j = std::get<1>(ij);
        return order == GridOrder::Col ? int(i % p + (j % q) * p) : int((i % p) * q + j % q);
    };
}

/// 1D block-cyclic process map over rows (Col) or columns (Row) (func.hh:207)
inline std::function<int(ij_tuple)> process_1d_grid(GridOrder order, int size) {
    return [order, size](ij_tuple ij) {
        return order == GridOrder::Col ? int(std::get<0>(ij) % size) : int(std::get<1>(ij) % size);
    };
}

/// device map: one device per process in this framework (func.hh:101-146)
inline std::function<int(ij_tuple)> device_1d_grid(GridOrder, int, int) {
    return [](ij_tuple) { return 0; };
}
inline std::function<int(ij_tuple)> device_2d_grid(GridOrder, int, int, int, int) {
    return [](ij_tuple) { return 0; };
}

/// transpose a tile map (func.hh:230)
template <typename F>
inline std::function<int(ij_tuple)> transpose_grid(F f) {
    return [f](ij_tuple ij) { return f(ij_tuple(std::get<1>(ij), std::get<0>(ij))); };
}

/// Detect whether a tile map is 2D cyclic; returns (order, p, q) (func.hh:265)
inline bool is_2d_cyclic_grid(int64_t mt, int64_t nt, std::function<int(ij_tuple)> f,
                              GridOrder* order, int* p, int* q) {
    // find p: first i > 0 with f(i,0) == f(0,0); q similarly
    int64_t pp = mt, qq = nt;
    for (int64_t i = 1; i < mt; ++i) if (f(ij_tuple(i, 0)) == f(ij_tuple(0, 0))) { pp = i; break; }
    for (int64_t j = 1; j < nt; ++j) if (f(ij_tuple(0, j)) == f(ij_tuple(0, 0))) { qq = j; break; }
    GridOrder o = (qq > 1 && pp > 1 && f(ij_tuple(1, 0)) == f(ij_tuple(0, 0)) + 1) ? GridOrder::Col
                : (pp > 1 ? GridOrder::Row : GridOrder::Col);
    if (pp == 1 && qq > 1) o = f(ij_tuple(0, 1)) == 1 ? GridOrder::Row : GridOrder::Col;
    auto g = process_2d_grid(o, int(pp), int(qq));
    for (int64_t j = 0; j < nt; ++j)
        for (int64_t i = 0; i < mt; ++i)
            if (g(ij_tuple(i, j)) != f(ij_tuple(i, j))) return false;
    if (order) *order = o;
    if (p) *p = int(pp);
    if (q) *q = int(qq);
    return true;
}

}  // namespace func
}  // namespace slate
