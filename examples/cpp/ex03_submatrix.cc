// ex03: sub-matrices by tile ranges and element slices (reference
// examples/ex03_submatrix.cc).  Views share storage with the parent.
#include "util.hh"

int main() {
    slate::init_grid();
    ex::banner("ex03_submatrix");
    int fails = 0;
    const int64_t m = 400, n = 320, nb = 64;
    slate::Matrix<double> A(m, n, nb);
    ex::random_fill(A, 3);
    auto o = ex::opts();

    auto B = A.sub(1, 3, 2, 4);                   // tiles [1..3] x [2..4]
    fails += ex::check("sub dims", double(B.m() != 3 * nb || B.n() != 3 * nb), 0);
    auto C = A.slice(10, 209, 5, 104);            // rows 10..209, cols 5..104
    fails += ex::check("slice dims", double(C.m() != 200 || C.n() != 100), 0);

    // zeroing the sub-matrix through the view changes the parent
    slate::set(0.0, 0.0, B, o);
    auto back = A.sub(1, 3, 2, 4);
    fails += ex::check("write through view", slate::norm(slate::Norm::Max, back, o), 0);
    // multiply two slices: sub-problem of a larger matrix, no copies
    slate::Matrix<double> D(200, 200, nb);
    D.insertLocalTiles(ex::target());
    auto X = A.slice(0, 99, 0, 199);
    slate::gemm(1.0, slate::conj_transpose(X), X, 0.0, D, o);   // D = X^T X (SPD-ish)
    fails += ex::check("gemm on slices ran", double(!(slate::norm(slate::Norm::Max, D, o) > 0)), 0);
    return ex::finish(fails);
}
