// Driver bindings, templated over the scalar type.
#pragma once

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include "slate_amd/slate.hh"
#include "slate_amd/local_blas.hh"
#include "slate_amd/eig_host.hh"
#include <pybind11/numpy.h>

namespace py = pybind11;

slate::Options to_options(py::dict d);

/// HIP queue of the direct local-kernel entry points (lb_*): 0 by default;
/// measurement scripts put them on the panel queue (1) with a background
/// GEMM on the trailing queue to time a factorization's critical path under
/// the contention the real run has (scripts/critpath.py --contended).
inline int& ops_queue() { static int q = 0; return q; }

template <typename T>
void bind_drivers(py::module_& m, std::string const& s) {
    using namespace slate;
    using R = real_type<T>;
    using G = py::call_guard<py::gil_scoped_release>;
    auto O = [](py::dict d) { return to_options(d); };
    (void)O;
#define DEF(name, ...) m.def((std::string(name) + "_" + s).c_str(), __VA_ARGS__)

    // ---- level 3 BLAS
    DEF("gemm", [](T a, Matrix<T> const& A, Matrix<T> const& B, T b, Matrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; gemm(a, A, B, b, C, op); });
    DEF("gemmA", [](T a, Matrix<T> const& A, Matrix<T> const& B, T b, Matrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; gemmA(a, A, B, b, C, op); });
    DEF("gemmC", [](T a, Matrix<T> const& A, Matrix<T> const& B, T b, Matrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; gemmC(a, A, B, b, C, op); });
    DEF("hemm", [](Side sd, T a, HermitianMatrix<T> const& A, Matrix<T> const& B, T b, Matrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; hemm(sd, a, A, B, b, C, op); });
    DEF("symm", [](Side sd, T a, SymmetricMatrix<T> const& A, Matrix<T> const& B, T b, Matrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; symm(sd, a, A, B, b, C, op); });
    DEF("herk", [](R a, Matrix<T> const& A, R b, HermitianMatrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; herk(a, A, b, C, op); });
    DEF("syrk", [](T a, Matrix<T> const& A, T b, SymmetricMatrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; syrk(a, A, b, C, op); });
    DEF("her2k", [](T a, Matrix<T> const& A, Matrix<T> const& B, R b, HermitianMatrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; her2k(a, A, B, b, C, op); });
    DEF("syr2k", [](T a, Matrix<T> const& A, Matrix<T> const& B, T b, SymmetricMatrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; syr2k(a, A, B, b, C, op); });
    DEF("trmm", [](Side sd, T a, TriangularMatrix<T> const& A, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; trmm(sd, a, A, B, op); });
    DEF("trsm", [](Side sd, T a, TriangularMatrix<T> const& A, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; trsm(sd, a, A, B, op); });

    // ---- aux
    DEF("add", [](T a, Matrix<T> const& A, T b, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; add(a, A, b, B, op); });
    DEF("tzadd", [](T a, BaseTrapezoidMatrix<T> const& A, T b, BaseTrapezoidMatrix<T>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; add(a, A, b, B, op); });
    DEF("copy", [](BaseMatrix<T> const& A, BaseMatrix<T>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; slate::copy<T, T>(A, B, op); });
    DEF("scale", [](R num, R den, BaseMatrix<T>& A, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; scale(num, den, A, op); });
    DEF("scale_row_col", [](Equed e, std::vector<R> const& Rv, std::vector<R> const& Cv, Matrix<T>& A, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; scale_row_col(e, Rv, Cv, A, op); });
    DEF("set", [](T off, T d, BaseMatrix<T>& A, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; set(off, d, A, op); });
    DEF("set_lambda", [](std::function<T(int64_t, int64_t)> f, BaseMatrix<T>& A, py::dict o) {
        Options op = to_options(o); set(f, A, op); });
    DEF("redistribute", [](Matrix<T> const& A, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; redistribute(A, B, op); });
    DEF("norm", [](Norm n, BaseMatrix<T> const& A, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; return norm(n, A, op); });
    DEF("colNorms", [](Norm n, Matrix<T> const& A, py::dict o) {
        Options op = to_options(o);
        std::vector<R> v(A.n());
        { py::gil_scoped_release r; colNorms(n, A, v.data(), op); }
        return v;
    });

    DEF("generate_matrix", [](std::string kind, BaseMatrix<T>& A, uint64_t seed, double shift, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; generate_matrix(kind, A, seed, shift, op); });
    // full generator (MatgenParams): returns (Sigma, cond_actual); sigma_in used by the _specified distribution
    DEF("matgen", [](std::string kind, Matrix<T>& A, int64_t seed, double cond, double condD,
                     std::vector<R> sigma_in, py::dict o) {
        Options op = to_options(o);
        MatgenParams p; p.kind = kind; p.seed = seed; p.cond_request = cond; p.condD = condD;
        std::vector<R> S = sigma_in;
        { py::gil_scoped_release r; generate_matrix(p, A, S, op); }
        return py::make_tuple(S, p.cond_actual);
    });
    DEF("matgen_tz", [](std::string kind, BaseTrapezoidMatrix<T>& A, int64_t seed, double cond, double condD,
                        py::dict o) {
        Options op = to_options(o);
        MatgenParams p; p.kind = kind; p.seed = seed; p.cond_request = cond; p.condD = condD;
        std::vector<R> S;
        { py::gil_scoped_release r; generate_matrix(p, A, S, op); }
        return py::make_tuple(S, p.cond_actual);
    });

    // ---- Cholesky
    DEF("potrf", [](HermitianMatrix<T>& A, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; return potrf(A, op); });

    DEF("potrs", [](HermitianMatrix<T>& A, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; potrs(A, B, op); });
    DEF("posv", [](HermitianMatrix<T>& A, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; return posv(A, B, op); });
    DEF("potri", [](HermitianMatrix<T>& A, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; return potri(A, op); });
    DEF("trtri", [](TriangularMatrix<T>& A, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; return trtri(A, op); });
    DEF("trtrm", [](TriangularMatrix<T>& A, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; trtrm(A, op); });

    // ---- LU (pivots as list of lists of (tile_index, offset))
    auto piv_out = [](Pivots const& P) {
        py::list out;
        for (auto const& v : P) {
            py::list l;
            for (auto const& x : v) l.append(py::make_tuple(x.tileIndex(), x.elementOffset()));
            out.append(l);
        }
        return out;
    };
    auto piv_in = [](py::list L) {
        Pivots P;
        for (auto v : L) {
            std::vector<Pivot> pv;
            for (auto x : v.cast<py::list>()) {
                auto t = x.cast<py::tuple>();
                pv.emplace_back(t[0].cast<int64_t>(), t[1].cast<int64_t>());
            }
            P.push_back(pv);
        }
        return P;
    };
    DEF("getrf", [=](Matrix<T>& A, py::dict o) {
        Options op = to_options(o); Pivots P; int64_t info;
        { py::gil_scoped_release r; info = getrf(A, P, op); }
        return py::make_tuple(info, piv_out(P)); });
    DEF("getrf_tntpiv", [=](Matrix<T>& A, py::dict o) {
        Options op = to_options(o); Pivots P; int64_t info;
        { py::gil_scoped_release r; info = getrf_tntpiv(A, P, op); }
        return py::make_tuple(info, piv_out(P)); });
    DEF("getrf_nopiv", [](Matrix<T>& A, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; return getrf_nopiv(A, op); });
    DEF("getrs", [=](Matrix<T> const& A, py::list piv, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); Pivots P = piv_in(piv); py::gil_scoped_release r; getrs(A, P, B, op); });
    DEF("getrs_op", [=](Op trans, Matrix<T> const& A, py::list piv, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); Pivots P = piv_in(piv); py::gil_scoped_release r; getrs(trans, A, P, B, op); });
    DEF("getrs_nopiv", [](Matrix<T> const& A, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; getrs_nopiv(A, B, op); });
    DEF("gesv", [=](Matrix<T>& A, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); Pivots P; int64_t info;
        { py::gil_scoped_release r; info = gesv(A, P, B, op); }
        return py::make_tuple(info, piv_out(P)); });
    DEF("gesv_nopiv", [](Matrix<T>& A, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; return gesv_nopiv(A, B, op); });
    DEF("getri", [=](Matrix<T>& A, py::list piv, py::dict o) {
        Options op = to_options(o); Pivots P = piv_in(piv); py::gil_scoped_release r; return getri(A, P, op); });
    if constexpr (std::is_same_v<T, double> || std::is_same_v<T, std::complex<double>>) {
        DEF("gesv_mixed", [=](Matrix<T>& A, Matrix<T>& B, Matrix<T>& X, py::dict o) {
            Options op = to_options(o); Pivots P; int iter = 0; int64_t info;
            { py::gil_scoped_release r; info = gesv_mixed(A, P, B, X, iter, op); }
            return py::make_tuple(info, piv_out(P), iter); });
        DEF("posv_mixed", [](HermitianMatrix<T>& A, Matrix<T>& B, Matrix<T>& X, py::dict o) {
            Options op = to_options(o); int iter = 0; int64_t info;
            { py::gil_scoped_release r; info = posv_mixed(A, B, X, iter, op); }
            return py::make_tuple(info, iter); });
        DEF("gesv_mixed_gmres", [=](Matrix<T>& A, Matrix<T>& B, Matrix<T>& X, py::dict o) {
            Options op = to_options(o); Pivots P; int iter = 0; int64_t info;
            { py::gil_scoped_release r; info = gesv_mixed_gmres(A, P, B, X, iter, op); }
            return py::make_tuple(info, piv_out(P), iter); });
        DEF("posv_mixed_gmres", [](HermitianMatrix<T>& A, Matrix<T>& B, Matrix<T>& X, py::dict o) {
            Options op = to_options(o); int iter = 0; int64_t info;
            { py::gil_scoped_release r; info = posv_mixed_gmres(A, B, X, iter, op); }
            return py::make_tuple(info, iter); });
    }
    DEF("gecondest", [](Norm nm, Matrix<T>& A, real_type<T> anorm, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; return gecondest(nm, A, anorm, op); });
    DEF("pocondest", [](Norm nm, HermitianMatrix<T>& A, real_type<T> anorm, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; return pocondest(nm, A, anorm, op); });
    DEF("trcondest", [](Norm nm, TriangularMatrix<T>& A, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; return trcondest(nm, A, op); });

    // ---- QR / LQ
    DEF("geqrf", [](Matrix<T>& A, py::dict o) {
        Options op = to_options(o); TriangularFactors<T> Tf;
        { py::gil_scoped_release r; geqrf(A, Tf, op); }
        return Tf; });
    DEF("gelqf", [](Matrix<T>& A, py::dict o) {
        Options op = to_options(o); TriangularFactors<T> Tf;
        { py::gil_scoped_release r; gelqf(A, Tf, op); }
        return Tf; });
    DEF("unmqr", [](Side sd, Op opq, Matrix<T> const& A, TriangularFactors<T> const& Tf, Matrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; unmqr(sd, opq, A, Tf, C, op); });
    DEF("unmlq", [](Side sd, Op opq, Matrix<T> const& A, TriangularFactors<T> const& Tf, Matrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; unmlq(sd, opq, A, Tf, C, op); });
    DEF("gels", [](Matrix<T>& A, Matrix<T>& BX, py::dict o) {
        Options op = to_options(o); TriangularFactors<T> Tf;
        { py::gil_scoped_release r; gels(A, Tf, BX, op); }
        return Tf; });
    DEF("cholqr", [](Matrix<T>& A, Matrix<T>& R, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; return cholqr(A, R, op); });

    DEF("getri_oop", [=](Matrix<T>& A, py::list piv, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); Pivots P = piv_in(piv); py::gil_scoped_release r; return getri(A, P, B, op); });
    DEF("gesv_rbt", [](Matrix<T>& A, Matrix<T>& B, Matrix<T>& X, py::dict o) {
        Options op = to_options(o); int iter = 0; int64_t info;
        { py::gil_scoped_release r; info = gesv_rbt(A, B, X, iter, op); }
        return py::make_tuple(info, iter); });
    DEF("gerbt", [](Matrix<T>& A, int depth, uint64_t su, uint64_t sv, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; gerbt(A, depth, su, sv, op); });
    // ---- band
    DEF("gbtrf", [=](BandMatrix<T>& A, py::dict o) {
        Options op = to_options(o); Pivots P; int64_t info;
        { py::gil_scoped_release r; info = gbtrf(A, P, op); }
        return py::make_tuple(info, piv_out(P)); });
    DEF("gbtrs", [=](BandMatrix<T> const& A, py::list piv, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); Pivots P = piv_in(piv); py::gil_scoped_release r; gbtrs(A, P, B, op); });
    DEF("gbsv", [=](BandMatrix<T>& A, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); Pivots P; int64_t info;
        { py::gil_scoped_release r; info = gbsv(A, P, B, op); }
        return py::make_tuple(info, piv_out(P)); });
    DEF("pbtrf", [](HermitianBandMatrix<T>& A, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; return pbtrf(A, op); });
    DEF("pbtrs", [](HermitianBandMatrix<T> const& A, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; pbtrs(A, B, op); });
    DEF("pbsv", [](HermitianBandMatrix<T>& A, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; return pbsv(A, B, op); });
    DEF("gbmm", [](T a, BandMatrix<T> const& A, Matrix<T> const& B, T b, Matrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; gbmm(a, A, B, b, C, op); });
    DEF("hbmm", [](Side sd, T a, HermitianBandMatrix<T> const& A, Matrix<T> const& B, T b, Matrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; hbmm(sd, a, A, B, b, C, op); });
    DEF("tbsm", [](Side sd, T a, TriangularBandMatrix<T> const& A, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; tbsm(sd, a, A, B, op); });
    DEF("tbsm_pivots", [piv_in](Side sd, T a, TriangularBandMatrix<T> const& A, py::list piv, Matrix<T>& B,
                                py::dict o) {
        Options op = to_options(o); Pivots P = piv_in(piv); py::gil_scoped_release r; tbsm(sd, a, A, P, B, op); });
    // ---- Hermitian indefinite (LAPACK-style ipiv list)
    DEF("hetrf", [](HermitianMatrix<T>& A, py::dict o) {
        Options op = to_options(o); std::vector<int64_t> ip; int64_t info;
        { py::gil_scoped_release r; info = hetrf(A, ip, op); }
        return py::make_tuple(info, ip); });
    DEF("hetrs", [](HermitianMatrix<T> const& A, std::vector<int64_t> ip, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; hetrs(A, ip, B, op); });
    DEF("hesv", [](HermitianMatrix<T>& A, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); std::vector<int64_t> ip; int64_t info;
        { py::gil_scoped_release r; info = hesv(A, ip, B, op); }
        return py::make_tuple(info, ip); });
    // ---- Aasen (reference signatures): T is a band matrix (kl = ku = nb) the caller provides
    DEF("hetrf_aasen", [=](HermitianMatrix<T>& A, BandMatrix<T>& Tb, py::dict o) {
        Options op = to_options(o); Pivots P, P2; Matrix<T> H; int64_t info;
        { py::gil_scoped_release r; info = hetrf(A, P, Tb, P2, H, op); }
        return py::make_tuple(info, piv_out(P), piv_out(P2)); });
    DEF("hetrs_aasen", [=](HermitianMatrix<T>& A, py::list piv, BandMatrix<T>& Tb, py::list piv2, Matrix<T>& B,
                           py::dict o) {
        Options op = to_options(o); Pivots P = piv_in(piv), P2 = piv_in(piv2);
        py::gil_scoped_release r; hetrs(A, P, Tb, P2, B, op); });
    DEF("hesv_aasen", [=](HermitianMatrix<T>& A, BandMatrix<T>& Tb, Matrix<T>& B, py::dict o) {
        Options op = to_options(o); Pivots P, P2; Matrix<T> H; int64_t info;
        { py::gil_scoped_release r; info = hesv(A, P, Tb, P2, H, B, op); }
        return py::make_tuple(info, piv_out(P), piv_out(P2)); });

    // ---- eigenvalues / SVD (None for an unwanted vector matrix)
    auto opt_mat = [](py::object z) { return z.is_none() ? Matrix<T>() : z.cast<Matrix<T>>(); };
    DEF("heev", [=](HermitianMatrix<T>& A, py::object z, py::dict o) {
        Options op = to_options(o); Matrix<T> Z = opt_mat(z); std::vector<R> L;
        { py::gil_scoped_release r; heev(A, L, Z, op); }
        return L; });
    DEF("hegv", [=](int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T>& B, py::object z, py::dict o) {
        Options op = to_options(o); Matrix<T> Z = opt_mat(z); std::vector<R> L;
        { py::gil_scoped_release r; hegv(itype, A, B, L, Z, op); }
        return L; });
    DEF("hegst", [](int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T> const& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; hegst(itype, A, B, op); });
    DEF("svd", [=](Matrix<T>& A, py::object u, py::object vt, py::dict o) {
        Options op = to_options(o); Matrix<T> U = opt_mat(u), VT = opt_mat(vt); std::vector<R> S;
        { py::gil_scoped_release r; svd(A, S, U, VT, op); }
        return S; });
    DEF("he2hb", [](Matrix<T>& A, py::dict o) {
        Options op = to_options(o); std::vector<TriangularFactors<T>> Ts;
        { py::gil_scoped_release r; he2hb(A, Ts, op); }
        return Ts; });
    DEF("ge2tb", [](Matrix<T>& A, py::dict o) {
        Options op = to_options(o); std::vector<TriangularFactors<T>> TU, TV;
        { py::gil_scoped_release r; ge2tb(A, TU, TV, op); }
        return py::make_tuple(TU, TV); });
    DEF("print", [](std::string label, BaseMatrix<T> const& A, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; return print_to_string(label.c_str(), A, op); });
    // ---- Debug (debug.hh)
    DEF("debug_print_tiles", [](BaseMatrix<T> const& A) { return Debug::printTiles(A); });
    DEF("debug_check_tiles_lives", [](BaseMatrix<T> const& A) { return Debug::checkTilesLives(A); });
    DEF("debug_check_tiles_layout", [](BaseMatrix<T> const& A) { return Debug::checkTilesLayout(A); });
    DEF("debug_diff_lapack", [](py::array_t<T, py::array::f_style | py::array::forcecast> a,
                                py::array_t<T, py::array::f_style | py::array::forcecast> b, int64_t mb, int64_t nb,
                                double tol) {
        slate_error_if_msg(a.ndim() != 2 || b.ndim() != 2 || a.shape(0) != b.shape(0) || a.shape(1) != b.shape(1),
                           "debug_diff_lapack: shapes differ");
        std::string map;
        int64_t nd = Debug::diffLapackMatrices<T>(a.shape(0), a.shape(1), a.data(), std::max<int64_t>(1, a.shape(0)),
                                                  b.data(), std::max<int64_t>(1, b.shape(0)), mb, nb, tol, &map);
        return py::make_tuple(nd, map); });
    // ---- stage-level two-stage API on distributed matrices (eig_stages.cc)
    py::class_<BandReflectors<T>>(m, ("BandReflectors_" + s).c_str())
        .def("size", [](BandReflectors<T> const& V) { return V.Q.size(); });
    DEF("hb2st_band", [](HermitianBandMatrix<T>& A, py::dict o) {
        Options op = to_options(o); std::vector<R> D, E; BandReflectors<T> V;
        { py::gil_scoped_release r; hb2st(A, D, E, V, op); }
        return py::make_tuple(D, E, V); });
    DEF("unmtr_hb2st", [](Side sd, Op op_, BandReflectors<T> const& V, Matrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; unmtr_hb2st(sd, op_, V, C, op); });
    DEF("unmtr_he2hb", [](Side sd, Op op_, Matrix<T>& A, std::vector<TriangularFactors<T>> Ts, Matrix<T>& C,
                          py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; unmtr_he2hb(sd, op_, A, Ts, C, op); });
    DEF("tb2bd_band", [](TriangularBandMatrix<T>& A, py::dict o) {
        Options op = to_options(o); std::vector<R> D, E; BandReflectors<T> U, V;
        { py::gil_scoped_release r; tb2bd(A, D, E, U, V, op); }
        return py::make_tuple(D, E, U, V); });
    DEF("unmbr_tb2bd", [](Side sd, Op op_, BandReflectors<T> const& V, Matrix<T>& C, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; unmbr_tb2bd(sd, op_, V, C, op); });
    DEF("unmbr_ge2tb", [](Side sd, Op op_, Matrix<T>& A, std::vector<TriangularFactors<T>> Ts, Matrix<T>& C,
                          py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; unmbr_ge2tb(sd, op_, A, Ts, C, op); });
    DEF("steqr2", [](Job jobz, std::vector<R> D, std::vector<R> E, Matrix<T>& Z, py::dict o) {
        Options op = to_options(o);
        { py::gil_scoped_release r; steqr2(jobz, D, E, Z, op); }
        return D; });
    DEF("bdsqr_mat", [=](Job ju, Job jv, std::vector<R> D, std::vector<R> E, py::object u, py::object vt,
                         py::dict o) {
        Options op = to_options(o); Matrix<T> U = opt_mat(u), VT = opt_mat(vt);
        { py::gil_scoped_release r; bdsqr(ju, jv, D, E, U, VT, op); }
        return D; });
    DEF("gels_cholqr", [](Matrix<T>& A, Matrix<T>& Rm, Matrix<T>& BX, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; gels_cholqr(A, Rm, BX, op); });
    DEF("gels_qr", [](Matrix<T>& A, Matrix<T>& BX, py::dict o) {
        Options op = to_options(o); TriangularFactors<T> Tf;
        { py::gil_scoped_release r; gels_qr(A, Tf, BX, op); }
        return Tf; });
    if constexpr (!is_complex_v<T>) {
        DEF("stedc_mat", [](std::vector<T> D, std::vector<T> E, Matrix<T>& Q, py::dict o) {
            Options op = to_options(o);
            { py::gil_scoped_release r; stedc(D, E, Q, op); }
            return D; });
        DEF("syev", [=](SymmetricMatrix<T>& A, py::object z, py::dict o) {
            Options op = to_options(o); Matrix<T> Z = opt_mat(z); std::vector<R> L;
            { py::gil_scoped_release r; syev(A, L, Z, op); }
            return L; });
        DEF("sygv", [=](int64_t itype, SymmetricMatrix<T>& A, SymmetricMatrix<T>& B, py::object z, py::dict o) {
            Options op = to_options(o); Matrix<T> Z = opt_mat(z); std::vector<R> L;
            { py::gil_scoped_release r; sygv(itype, A, B, L, Z, op); }
            return L; });
        DEF("sysv", [](SymmetricMatrix<T>& A, Matrix<T>& B, py::dict o) {
            Options op = to_options(o); std::vector<int64_t> ip; int64_t info;
            { py::gil_scoped_release r; info = sysv(A, ip, B, op); }
            return py::make_tuple(info, ip); });
    }

    // host stage-2 kernels on dense numpy arrays (column-major copies)
    DEF("hb2st", [](py::array_t<T, py::array::f_style | py::array::forcecast> a, int64_t kd) {
        auto b = a.request();
        int64_t n = b.shape[0];
        std::vector<T> A((T*)b.ptr, (T*)b.ptr + n * n);
        std::vector<R> d, e; host::Reflectors<T> Q; std::vector<T> ph;
        { py::gil_scoped_release r; host::hb2st<T>(n, kd, A.data(), n, d, e, Q, ph); }
        return py::make_tuple(d, e); });
    DEF("tb2bd", [](py::array_t<T, py::array::f_style | py::array::forcecast> a, int64_t kd) {
        auto b = a.request();
        int64_t m = b.shape[0], n = b.shape[1];
        std::vector<T> A((T*)b.ptr, (T*)b.ptr + m * n);
        std::vector<R> d, e; host::Reflectors<T> QU, QV; std::vector<T> pu, pv;
        { py::gil_scoped_release r; host::tb2bd<T>(m, n, kd, A.data(), m, d, e, QU, QV, pu, pv); }
        return py::make_tuple(d, e); });

    // ---- direct local-kernel access on raw device pointers (single process)
    auto dctx = []() { return lb::Ctx::device(ops_queue()); };
    auto dsync = [](lb::Ctx const& c) { slate_hip_call(hipStreamSynchronize(c.stream)); };
    auto cop = [](std::string const& x) { return x == "N" ? Op::NoTrans : x == "T" ? Op::Trans : Op::ConjTrans; };
    auto cup = [](std::string const& x) { return x == "L" ? Uplo::Lower : x == "U" ? Uplo::Upper : Uplo::General; };
    // background GEMM: launched on `queue`, not waited for (queue_sync(queue))
    DEF("lb_gemm_async", [=](int queue, std::string ta, std::string tb, int64_t mm, int64_t n, int64_t k, T a,
                             uintptr_t A, int64_t lda, uintptr_t B, int64_t ldb, T b, uintptr_t C, int64_t ldc) {
        py::gil_scoped_release r;
        lb::gemm<T>(lb::Ctx::device(queue), cop(ta), cop(tb), mm, n, k, a, (T const*)A, lda, (T const*)B, ldb, b,
                    (T*)C, ldc);
    });
    DEF("lb_gemm", [=](std::string ta, std::string tb, int64_t mm, int64_t n, int64_t k, T a, uintptr_t A, int64_t lda,
                       uintptr_t B, int64_t ldb, T b, uintptr_t C, int64_t ldc) {
        py::gil_scoped_release r;
        auto c = dctx();
        lb::gemm<T>(c, cop(ta), cop(tb), mm, n, k, a, (T*)A, lda, (T*)B, ldb, b, (T*)C, ldc);
        dsync(c);
    });
    DEF("lb_herk", [=](std::string up, std::string op, int64_t n, int64_t k, R a, uintptr_t A, int64_t lda, R b,
                       uintptr_t C, int64_t ldc) {
        py::gil_scoped_release r;
        auto c = dctx();
        lb::herk<T>(c, cup(up), cop(op), n, k, a, (T*)A, lda, b, (T*)C, ldc);
        dsync(c);
    });
    DEF("lb_trsm", [=](std::string sd, std::string up, std::string op, std::string dg, int64_t mm, int64_t n, T a,
                       uintptr_t A, int64_t lda, uintptr_t B, int64_t ldb) {
        py::gil_scoped_release r;
        auto c = dctx();
        lb::trsm<T>(c, sd == "L" ? Side::Left : Side::Right, cup(up), cop(op), dg == "U" ? Diag::Unit : Diag::NonUnit,
                    mm, n, a, (T*)A, lda, (T*)B, ldb);
        dsync(c);
    });
    DEF("lb_potrf", [=](std::string up, int64_t n, uintptr_t A, int64_t lda) {
        py::gil_scoped_release r;
        auto c = dctx();
        device::Buffer<int> info(1);
        device::memset_async(info.data(), 0, sizeof(int), c.stream);
        lb::potrf<T>(c, cup(up), n, (T*)A, lda, info.data(), 0);
        int h = 0;
        device::memcpy_async(&h, info.data(), sizeof(int), c.stream);
        dsync(c);
        return h;
    });
    DEF("lb_lu_sign", [=](int64_t n, uintptr_t A, int64_t lda) {
        // sign-modified LU of the Householder reconstruction (lu_dist.cc):
        // L U = A + diag(s); returns s
        std::vector<T> h(std::max<int64_t>(n, 0));
        {
            py::gil_scoped_release r;
            auto c = dctx();
            device::Buffer<T> sgn(n + 1);
            internal::ludist::lu_sign<T>(c, n, (T*)A, lda, sgn.data());
            if (n > 0) device::memcpy_async(h.data(), sgn.data(), sizeof(T) * size_t(n), c.stream);
            dsync(c);
        }
        return h;
    });
    DEF("lb_getrf_panel", [=](int64_t mm, int64_t n, uintptr_t A, int64_t lda, bool tournament) {
        std::vector<int64_t> ipiv(std::min(mm, n));
        int h = 0;
        {
            py::gil_scoped_release r;
            auto c = dctx();
            device::Buffer<int> info(1);
            device::Buffer<int64_t> dpiv(ipiv.size() + 1), perm(mm + 1);
            device::memset_async(info.data(), 0, sizeof(int), c.stream);
            lb::getrf_panel<T>(c, mm, n, (T*)A, lda, dpiv.data(), perm.data(), info.data(), 0, true, tournament);
            device::memcpy_async(ipiv.data(), dpiv.data(), ipiv.size() * sizeof(int64_t), c.stream);
            device::memcpy_async(&h, info.data(), sizeof(int), c.stream);
            dsync(c);
        }
        return py::make_tuple(h, ipiv);
    });
    DEF("lb_geqrf_panel", [=](int64_t mm, int64_t n, uintptr_t A, int64_t lda) {
        int64_t k = std::min(mm, n);
        std::vector<T> tau(k), Tm(k * k);
        {
            py::gil_scoped_release r;
            auto c = dctx();
            device::Buffer<T> dt(k + 1), dT(k * k + 1);
            lb::geqrf_panel<T>(c, mm, n, (T*)A, lda, dt.data(), dT.data(), k);
            device::memcpy_async(tau.data(), dt.data(), k * sizeof(T), c.stream);
            device::memcpy_async(Tm.data(), dT.data(), k * k * sizeof(T), c.stream);
            dsync(c);
        }
        return py::make_tuple(tau, Tm);
    });

#undef DEF
}

inline void bind_mixed(py::module_& m) {
    using namespace slate;
    m.def("copy_d2s", [](BaseMatrix<double> const& A, BaseMatrix<float>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; slate::copy<double, float>(A, B, op); });
    m.def("copy_s2d", [](BaseMatrix<float> const& A, BaseMatrix<double>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; slate::copy<float, double>(A, B, op); });
    m.def("copy_z2c", [](BaseMatrix<std::complex<double>> const& A, BaseMatrix<std::complex<float>>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; slate::copy<std::complex<double>, std::complex<float>>(A, B, op); });
    m.def("copy_c2z", [](BaseMatrix<std::complex<float>> const& A, BaseMatrix<std::complex<double>>& B, py::dict o) {
        Options op = to_options(o); py::gil_scoped_release r; slate::copy<std::complex<float>, std::complex<double>>(A, B, op); });
}
