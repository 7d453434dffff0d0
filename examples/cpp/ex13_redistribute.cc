// ex13: changing the tiling and the distribution of a matrix (reference
// examples/ex13_non_uniform_block_size.cc changes tile sizes per tile).
// Here matrices use uniform tiles (the local array is ScaLAPACK-layout, one
// contiguous block per GPU); different tilings, grids and source ranks are
// converted by redistribute / copy, and every driver accepts any of them.
#include "util.hh"

int main() {
    auto g = slate::init_grid();
    ex::banner("ex13_redistribute");
    int fails = 0;
    const int64_t n = 333;
    auto o = ex::opts();
    slate::Matrix<double> A(n, n, 64, g);
    ex::random_fill(A, 25);
    // same data, tile size 48, first tile on the last process row/column
    slate::Matrix<double> B(n, n, 48, 48, g, g->p() - 1, g->q() - 1);
    B.insertLocalTiles(ex::target());
    slate::redistribute(A, B, o);
    // and on the transposed grid with 80 x 40 tiles
    slate::Matrix<double> C(n, n, 80, 40, g->transposed());
    C.insertLocalTiles(ex::target());
    slate::copy<double, double>(B, C, o);
    fails += ex::check("norms agree after redistribution",
                       std::abs(slate::norm(slate::Norm::Fro, A, o) - slate::norm(slate::Norm::Fro, C, o)), 1e-9);
    // a solve on the redistributed copy matches the original
    slate::Matrix<double> X(n, 2, 48, 48, g, g->p() - 1, 0);
    ex::random_fill(X, 26);
    auto X0 = ex::copy_of(X), B0 = ex::copy_of(B);
    slate::set(0.0, double(n), B, o);   // make it diagonally dominant: B = n I + A
    slate::Matrix<double> Ar = B.emptyLike();
    Ar.insertLocalTiles(ex::target());
    slate::redistribute(A, Ar, o);
    slate::add(1.0, Ar, 1.0, B, o);
    auto Bs = ex::copy_of(B);
    int64_t info = slate::lu_solve(B, X, o);
    fails += ex::check("lu_solve on a 48x48-tiled, shifted-source matrix", info ? 1.0 : ex::solve_residual(Bs, X, X0), 1e-15);
    (void)B0;
    return ex::finish(fails);
}
