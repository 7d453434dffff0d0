// ex01: creating distributed matrices (reference examples/ex01_matrix.cc):
// empty matrices with allocated local storage, wrapping a LAPACK array
// (1 x 1), wrapping ScaLAPACK local arrays (p x q), emptyLike, element access.
#include "util.hh"
#include <vector>

int main() {
    slate::init_grid();
    ex::banner("ex01_matrix");
    auto g = slate::default_grid();
    int fails = 0;
    const int64_t m = 500, n = 300, nb = 64;

    // 1. library-allocated storage, 2D block-cyclic over the p x q grid
    slate::Matrix<double> A(m, n, nb, g);
    A.insertLocalTiles(ex::target());
    ex::random_fill(A, 1);
    fails += ex::check("A: dims / tile counts", double(A.m() != m || A.n() != n || A.mt() != 8 || A.nt() != 5), 0);

    // 2. user-owned ScaLAPACK local array: (numroc x numroc) column-major
    int64_t mloc = slate::numroc(m, nb, g->myrow(), g->p()), nloc = slate::numroc(n, nb, g->mycol(), g->q());
    std::vector<double> local(size_t(std::max<int64_t>(mloc, 1)) * std::max<int64_t>(nloc, 1));
    auto S = slate::Matrix<double>::fromScaLAPACK(m, n, local.data(), std::max<int64_t>(mloc, 1), nb, nb, g);
    slate::copy<double, double>(A, S, ex::opts());
    S.tileUpdateAllOrigin();   // make the user array authoritative again
    double diff = 0;
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < m; ++i)
            if (S.tileIsLocal(i / nb, j / nb)) diff = std::max(diff, std::abs(S.elem(i, j) - A.elem(i, j)));
    fails += ex::check("fromScaLAPACK copy", diff, 0);

    // 3. a LAPACK array on every rank (1 x 1 self grid view)
    std::vector<float> lap(size_t(64) * 64, 1.0f);
    auto L = slate::Matrix<float>::fromLAPACK(64, 64, lap.data(), 64, 16);
    fails += ex::check("fromLAPACK 1x1 owns all tiles", double(!L.tileIsLocal(3, 3)), 0);

    // 4. emptyLike: same shape and distribution, no data
    auto E = A.emptyLike();
    E.insertLocalTiles(ex::target());
    fails += ex::check("emptyLike distribution", double(E.tileRank(3, 2) != A.tileRank(3, 2)), 0);

    slate::print("A", A, {{slate::Option::PrintEdgeItems, int64_t(3)}});
    return ex::finish(fails);
}
