// Native command-line tester and benchmark (reference test/test.cc and
// test/test_*.cc): for each routine x type x dim x nb
// it generates grid-independent test matrices, times the driver between a
// barrier + device synchronization (MAX over ranks), and checks the result
// with DISTRIBUTED backward-error residuals (no gather of the operands, so the
// check scales with the run):
//   BLAS-3:   C X == op-expression applied to X, X random (reference test_gemm.cc:138-211)
//   solvers:  ||B - A X||_1 / (n ||A||_1 ||X||_1)         (test_gesv.cc:330-377)
//   QR / LQ:  ||A - Q R||_1 / (m ||A||_1)                  (test_geqrf.cc:155-216)
//   eig/svd:  ||A Z - Z Lambda||_1 / (n ||A||_1), ||A - U S V^H||_1 / (n ||A||_1)
// and reports "error <= tol * eps" as pass / FAILED, one table row per case.
//
//   slate_tester gemm,potrf,getrf --type d,z --dim 1000:4000:1000 --nb 256 --target d
//   python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
//       bin/slate_tester getrf_tntpiv --dim 65536 --nb 512 --grid 2x4 --check n
#include "slate_amd/slate.hh"
#include "slate_amd/trace.hh"

#include <array>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <sstream>
#include <string>
#include <vector>

using namespace slate;

namespace {

struct Params {
    std::string types = "d";
    std::vector<std::array<int64_t, 3>> dims{{500, 500, 500}};
    std::vector<int64_t> nbs{256};
    int p = 0, q = 0;
    Target target = device::available() ? Target::Devices : Target::HostTask;
    int64_t lookahead = 1;
    int64_t nrhs = 10;
    bool check = true;
    double tol = 50;
    int repeat = 1;
    bool trace = false;
    std::string matrix;          // --matrix: matgen kind of the main operand (default per routine)
    int64_t method_lu = -1, method_trsm = -1, method_gemm = -1, method_hemm = -1, method_cholqr = -1;
    char origin = 'x';           // --origin h|d: where the operands are generated (x: the target)
    int timer_level = 1;         // --timer-level 2: per-driver trace timers after each case
    int64_t itermax = -1;
    int fallback = -1;
    double pivot_threshold = -1;
    // operand shape flags of the BLAS-3 / triangular routines (reference
    // --uplo --trans --side --diag)
    Uplo uplo = Uplo::Lower;
    Op trans = Op::NoTrans;
    Side side = Side::Left;
    Diag diag = Diag::NonUnit;
    double cond = std::numeric_limits<double>::quiet_NaN();   // --cond: spectral --matrix kinds
    int64_t ib = -1;                                          // --ib: inner blocking
    bool nonuniform = false;                                  // --nonuniform-nb y: varying tile sizes
    GridOrder order = GridOrder::Col;                         // --go c|r: process grid order
    char dev_order = 'r';                                     // --do: one GPU per process (accepted)
};

std::vector<int64_t> parse_list(std::string const& s) {
    std::vector<int64_t> out;
    std::stringstream ss(s);
    std::string part;
    while (std::getline(ss, part, ',')) {
        size_t c1 = part.find(':');
        if (c1 == std::string::npos) { out.push_back(std::stoll(part)); continue; }
        size_t c2 = part.find(':', c1 + 1);
        int64_t a = std::stoll(part.substr(0, c1));
        int64_t b = std::stoll(part.substr(c1 + 1, c2 == std::string::npos ? std::string::npos : c2 - c1 - 1));
        int64_t st = c2 == std::string::npos ? a : std::stoll(part.substr(c2 + 1));
        for (int64_t v = a; v <= b; v += st) out.push_back(v);
    }
    return out;
}

std::vector<std::array<int64_t, 3>> parse_dims(std::string const& s) {
    std::vector<std::array<int64_t, 3>> out;
    std::stringstream ss(s);
    std::string part;
    while (std::getline(ss, part, ',')) {
        if (part.find('x') != std::string::npos) {
            std::vector<int64_t> v;
            std::stringstream ps(part);
            std::string t;
            while (std::getline(ps, t, 'x')) v.push_back(std::stoll(t));
            out.push_back({v[0], v.size() > 1 ? v[1] : v[0], v.size() > 2 ? v[2] : (v.size() > 1 ? v[1] : v[0])});
        } else {
            for (int64_t n : parse_list(part)) out.push_back({n, n, n});
        }
    }
    return out;
}

int rank() { return default_grid()->rank(); }

template <typename T>
using R_ = real_type<T>;

/// One test case: matrices on the default grid, options, timing helpers.
template <typename T>
struct Case {
    Params const& P;
    int64_t m, n, k, nb;
    uint64_t seed = 1;
    Options opts;
    Case(Params const& p, std::array<int64_t, 3> d, int64_t nb_)
        : P(p), m(d[0]), n(d[1]), k(d[2]), nb(nb_) {
        opts = {{Option::Target, P.target}, {Option::Lookahead, P.lookahead}};
        if (P.method_lu >= 0) opts[Option::MethodLU] = P.method_lu;
        if (P.method_cholqr >= 0) opts[Option::MethodCholQR] = P.method_cholqr;
        if (P.method_trsm >= 0) opts[Option::MethodTrsm] = P.method_trsm;
        if (P.method_gemm >= 0) opts[Option::MethodGemm] = P.method_gemm;
        if (P.method_hemm >= 0) opts[Option::MethodHemm] = P.method_hemm;
        if (P.itermax >= 0) opts[Option::MaxIterations] = P.itermax;
        if (P.fallback >= 0) opts[Option::UseFallbackSolver] = int64_t(P.fallback);
        if (P.pivot_threshold > 0) opts[Option::PivotThreshold] = P.pivot_threshold;
        if (P.ib > 0) opts[Option::InnerBlocking] = P.ib;
    }
    /// where operands are generated: --origin h puts them on the host (the
    /// drivers then move them to the target and back, reference --origin)
    Target gen_target() const {
        return P.origin == 'h' ? Target::HostTask : (P.origin == 'd' ? Target::Devices : P.target);
    }
    Matrix<T> mat(int64_t rows, int64_t cols, const char* kind = "rands", double shift = -1, bool main = false) {
        Matrix<T> A(rows, cols, nb, default_grid());
        const Target gt = gen_target();
        A.insertLocalTiles(gt);
        BaseMatrix<T>& b = A;
        Options go = opts;
        go[Option::Target] = gt;
        if (main && P.nonuniform) {
            // --nonuniform-nb: tiles alternate nb and nb/2 + 1 rows/cols, on a
            // 2-D cyclic tile map (the drivers' arbitrary-layout path)
            auto g = default_grid();
            const int64_t b0 = nb, b1 = std::max<int64_t>(1, nb / 2 + 1);
            auto tsz = [b0, b1](int64_t i) { return (i % 2 == 0) ? b0 : b1; };
            const int p = g->p(), q = g->q();
            const bool colmajor = P.order == GridOrder::Col;
            Matrix<T> An(rows, cols, tsz, tsz,
                         [p, q, colmajor](std::tuple<int64_t, int64_t> ij) {
                             const int64_t i = std::get<0>(ij) % p, j = std::get<1>(ij) % q;
                             return int(colmajor ? i + j * p : i * q + j);
                         },
                         [](std::tuple<int64_t, int64_t>) { return 0; }, g);
            An.insertLocalTiles(gt);
            BaseMatrix<T>& bn = An;
            generate_matrix(P.matrix.empty() ? std::string(kind) : P.matrix, bn, seed++, shift, go);
            return An;
        }
        if (main && !P.matrix.empty()) {
            // --matrix: any matgen kind (element kinds, or spectral ones such as
            // svd / poev / geev, whose condition number --cond sets)
            bool done = false;
            if (std::isnan(P.cond)) {
                try {
                    generate_matrix(P.matrix, b, seed, shift, go);
                    done = true;
                } catch (std::exception const&) {
                }
            }
            if (!done) {
                MatgenParams mp;
                mp.kind = P.matrix;
                mp.seed = int64_t(seed);
                mp.cond_request = P.cond;
                generate_matrix(mp, A, go);
            }
            ++seed;
            return A;
        }
        generate_matrix(std::string(kind), b, seed++, shift, go);
        return A;
    }
    Matrix<T> zeros(int64_t rows, int64_t cols) {
        Matrix<T> A(rows, cols, nb, default_grid());
        A.insertLocalTiles(P.target);
        set(T(0), T(0), A, opts);
        return A;
    }
    Matrix<T> copy_of(BaseMatrix<T> const& A) {
        Matrix<T> B(A.m(), A.n(), nb, default_grid());
        B.insertLocalTiles(P.target);
        copy<T, T>(A, B, opts);
        return B;
    }
    double nrm(BaseMatrix<T> const& A) { return double(norm(Norm::One, A, opts)); }
    /// seconds, MAX over ranks, bracketed by barrier + device sync
    double timed(std::function<void()> f) {
        auto& w = default_grid()->world();
        slate::sync();
        w.barrier();
        auto t0 = std::chrono::steady_clock::now();
        f();
        slate::sync();
        w.barrier();
        double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return w.allreduce_scalar<double>(t, ReduceOp::Max);
    }
    /// ||B0 - A X||_1 / (n ||A||_1 ||X||_1) for a general A
    double solve_resid(Matrix<T> const& A0, Matrix<T> const& X, Matrix<T> const& B0) {
        auto Rm = copy_of(B0);
        gemm(T(-1), A0, X, T(1), Rm, opts);
        return nrm(Rm) / (double(A0.n()) * nrm(A0) * nrm(X));
    }
};

struct Result { double time = NAN, error = NAN; double flops = 0; bool skipped = false; std::string note; };

template <typename T> double cfac() { return is_complex_v<T> ? 4.0 : 1.0; }
template <typename T> double gemm_fl(double m, double n, double k) { return cfac<T>() * 2 * m * n * k; }

//------------------------------------------------------------------------------
// Routines
template <typename T>
Result r_gemm(Case<T>& c) {
    auto A = c.mat(c.m, c.k), B = c.mat(c.k, c.n), C = c.mat(c.m, c.n);
    auto C0 = c.copy_of(C);
    T alpha(1.5), beta(-0.5);
    Result r;
    r.time = c.timed([&] { gemm(alpha, A, B, beta, C, c.opts); });
    r.flops = gemm_fl<T>(c.m, c.n, c.k);
    if (c.P.check) {
        auto X = c.mat(c.n, 4), BX = c.zeros(c.k, 4), CX = c.zeros(c.m, 4), Y = c.zeros(c.m, 4);
        gemm(T(1), C, X, T(0), CX, c.opts);          // C X
        gemm(T(1), B, X, T(0), BX, c.opts);
        gemm(T(1), C0, X, T(0), Y, c.opts);
        gemm(alpha, A, BX, beta, Y, c.opts);         // alpha A (B X) + beta C0 X
        add(T(-1), CX, T(1), Y, c.opts);
        r.error = c.nrm(Y) / ((std::abs(alpha) * c.nrm(A) * c.nrm(B) + std::abs(beta) * c.nrm(C0)) * c.nrm(X));
    }
    return r;
}

template <typename T>
Result r_herk(Case<T>& c) {
    auto A = c.mat(c.n, c.k), Cg = c.mat(c.n, c.n, "spd", 0.0);
    auto C0g = c.copy_of(Cg);
    HermitianMatrix<T> C(Uplo::Lower, Cg), C0(Uplo::Lower, C0g);
    R_<T> alpha(2), beta(-1);
    Result r;
    r.time = c.timed([&] { herk(alpha, A, beta, C, c.opts); });
    r.flops = cfac<T>() * double(c.k) * c.n * (c.n + 1);
    if (c.P.check) {
        auto X = c.mat(c.n, 4), CX = c.zeros(c.n, 4), Y = c.zeros(c.n, 4), AX = c.zeros(c.k, 4);
        hemm(Side::Left, T(1), C, X, T(0), CX, c.opts);
        hemm(Side::Left, T(beta), C0, X, T(0), Y, c.opts);
        gemm(T(1), conj_transpose(A), X, T(0), AX, c.opts);
        gemm(T(alpha), A, AX, T(1), Y, c.opts);
        add(T(-1), CX, T(1), Y, c.opts);
        r.error = c.nrm(Y) / ((double(alpha) * c.nrm(A) * c.nrm(A) + std::abs(double(beta)) * c.nrm(C0g)) * c.nrm(X));
    }
    return r;
}

template <typename T>
Result r_hemm(Case<T>& c) {
    auto Ag = c.mat(c.m, c.m, "spd", 0.0), B = c.mat(c.m, c.n), C = c.mat(c.m, c.n);
    auto C0 = c.copy_of(C);
    HermitianMatrix<T> A(Uplo::Lower, Ag);
    T alpha(1), beta(0.5);
    Result r;
    r.time = c.timed([&] { hemm(Side::Left, alpha, A, B, beta, C, c.opts); });
    r.flops = gemm_fl<T>(c.m, c.n, c.m);
    if (c.P.check) {
        auto X = c.mat(c.n, 4), CX = c.zeros(c.m, 4), BX = c.zeros(c.m, 4), Y = c.zeros(c.m, 4);
        gemm(T(1), C, X, T(0), CX, c.opts);
        gemm(T(1), B, X, T(0), BX, c.opts);
        gemm(beta, C0, X, T(0), Y, c.opts);
        hemm(Side::Left, alpha, A, BX, T(1), Y, c.opts);
        add(T(-1), CX, T(1), Y, c.opts);
        r.error = c.nrm(Y) / ((c.nrm(Ag) * c.nrm(B) + std::abs(beta) * c.nrm(C0)) * c.nrm(X));
    }
    return r;
}

/// dense diagonal part of a square matrix (a kl = ku = 0 band through gbmm)
template <typename T>
Matrix<T> dense_diag(Case<T>& c, Matrix<T> const& D) {
    auto I = c.zeros(D.n(), D.n()), F = c.zeros(D.m(), D.n());
    set(T(0), T(1), I, c.opts);
    gbmm(T(1), BandMatrix<T>(0, 0, D), I, T(0), F, c.opts);
    return F;
}

/// op(A) for --trans n|t|c on a triangular view
template <typename T>
TriangularMatrix<T> op_tri(Op op, TriangularMatrix<T> const& A) {
    if (op == Op::Trans) return transpose(A);
    if (op == Op::ConjTrans) return conj_transpose(A);
    return A;
}

template <typename T>
Result r_trsm(Case<T>& c) {
    // op(A) X = alpha B (--side l) or X op(A) = alpha B (--side r)
    const bool left = c.P.side == Side::Left;
    const int64_t an = left ? c.m : c.n;
    auto Tg = c.mat(an, an, "rands+n"), B = c.mat(c.m, c.n);
    auto B0 = c.copy_of(B);
    TriangularMatrix<T> A0(c.P.uplo, c.P.diag, Tg);
    auto A = op_tri(c.P.trans, A0);
    T alpha(2);
    Result r;
    r.time = c.timed([&] { trsm(c.P.side, alpha, A, B, c.opts); });
    r.flops = cfac<T>() * double(an) * an * (left ? c.n : c.m);
    if (c.P.check) {
        auto X = c.copy_of(B);
        trmm(c.P.side, T(1), A, X, c.opts);            // op(A) X  or  X op(A)
        add(-alpha, B0, T(1), X, c.opts);              //  - alpha B0
        r.error = c.nrm(X) / (c.nrm(Tg) * c.nrm(B) * double(an));
    }
    return r;
}

template <typename T>
Result r_trmm(Case<T>& c) {
    const bool left = c.P.side == Side::Left;
    const int64_t an = left ? c.m : c.n;
    auto Tg = c.mat(an, an, "rands+n"), B = c.mat(c.m, c.n);
    auto B0 = c.copy_of(B);
    TriangularMatrix<T> A0(c.P.uplo, c.P.diag, Tg);
    auto A = op_tri(c.P.trans, A0);
    Result r;
    r.time = c.timed([&] { trmm(c.P.side, T(1), A, B, c.opts); });
    r.flops = cfac<T>() * double(an) * an * (left ? c.n : c.m);
    if (c.P.check) {
        // forward check against a dense copy of the triangle: op(D) B0 or B0 op(D)
        // (a trsm back-substitution would be ill-conditioned for unit diagonals)
        auto D = c.zeros(an, an);
        BaseTrapezoidMatrix<T> Ts(c.P.uplo, Tg, MatrixKind::Trapezoid), Ds(c.P.uplo, D, MatrixKind::Trapezoid);
        copy<T, T>(Ts, Ds, c.opts);
        if (c.P.diag == Diag::Unit) {
            auto Dd = dense_diag(c, D);
            add(T(-1), Dd, T(1), D, c.opts);
            auto I = c.zeros(an, an);
            set(T(0), T(1), I, c.opts);
            add(T(1), I, T(1), D, c.opts);
        }
        Matrix<T> opD = c.P.trans == Op::Trans ? transpose(D) : (c.P.trans == Op::ConjTrans ? conj_transpose(D) : D);
        if (left) gemm(T(-1), opD, B0, T(1), B, c.opts);
        else gemm(T(-1), B0, opD, T(1), B, c.opts);
        r.error = c.nrm(B) / (c.nrm(D) * c.nrm(B0) * double(an));
    }
    return r;
}

// factor / solve family: run(A, B) factors and solves in place, residual vs A0
template <typename T>
Result solve_case(Case<T>& c, const char* kind, std::function<int64_t(Matrix<T>&, Matrix<T>&)> run,
                  double flops) {
    auto A = c.mat(c.n, c.n, kind, -1, true), B = c.mat(c.n, c.P.nrhs);
    auto A0 = c.copy_of(A), B0 = c.copy_of(B);
    Result r;
    int64_t info = 0;
    r.time = c.timed([&] { info = run(A, B); });
    r.flops = flops;
    if (info != 0) { r.error = INFINITY; r.note = "info=" + std::to_string(info); return r; }
    if (c.P.check) r.error = c.solve_resid(A0, B, B0);
    return r;
}

template <typename T> double getrf_fl(double n) { return cfac<T>() * (2.0 / 3 * n * n * n - 0.5 * n * n + 5.0 / 6 * n); }
template <typename T> double potrf_fl(double n) { return cfac<T>() * (n * n * n / 3 + n * n / 2 + n / 6); }

/// factorization timed alone; the solve for the check runs afterwards
template <typename T>
Result r_getrf_m(Case<T>& c, int64_t method) {
    auto A = c.mat(c.n, c.n, "rands", -1, true), B = c.mat(c.n, c.P.nrhs);
    auto A0 = c.copy_of(A), B0 = c.copy_of(B);
    Pivots piv;
    Options o = c.opts;
    if (c.P.method_lu < 0) o[Option::MethodLU] = method;
    Result r;
    int64_t info = 0;
    r.time = c.timed([&] { info = getrf(A, piv, o); });
    r.flops = getrf_fl<T>(c.n);
    if (info) { r.error = INFINITY; r.note = "info=" + std::to_string(info); return r; }
    if (c.P.check) {
        getrs(A, piv, B, c.opts);
        r.error = c.solve_resid(A0, B, B0);
    }
    return r;
}

template <typename T>
Result r_getrf_nopiv(Case<T>& c) {
    auto A = c.mat(c.n, c.n, "rands+n"), B = c.mat(c.n, c.P.nrhs);
    auto A0 = c.copy_of(A), B0 = c.copy_of(B);
    Result r;
    int64_t info = 0;
    r.time = c.timed([&] { info = getrf_nopiv(A, c.opts); });
    r.flops = getrf_fl<T>(c.n);
    if (info) { r.error = INFINITY; return r; }
    if (c.P.check) {
        getrs_nopiv(A, B, c.opts);
        r.error = c.solve_resid(A0, B, B0);
    }
    return r;
}

template <typename T>
Result r_gesv(Case<T>& c) {
    return solve_case<T>(c, "rands", [&](Matrix<T>& A, Matrix<T>& B) { Pivots piv; return gesv(A, piv, B, c.opts); },
                         getrf_fl<T>(c.n) + cfac<T>() * 2.0 * c.n * c.n * c.P.nrhs);
}

template <typename T>
Result r_gesv_mixed_v(Case<T>& c, int variant) {
    if constexpr (!std::is_same_v<T, double> && !std::is_same_v<T, std::complex<double>>) {
        Result r; r.skipped = true; r.note = "double precisions only"; return r;
    } else {
        const int64_t nrhs = (variant == 1 || variant == 3) ? 1 : c.P.nrhs;   // GMRES-IR: one right-hand side
        auto A = c.mat(c.n, c.n, variant >= 2 ? "spd" : "rands+n"), B = c.mat(c.n, nrhs);
        auto A0 = c.copy_of(A), X = c.zeros(c.n, nrhs);
        Result r;
        int64_t info = 0;
        int iter = 0;
        r.time = c.timed([&] {
            Pivots piv;
            if (variant == 0) info = gesv_mixed(A, piv, B, X, iter, c.opts);
            else if (variant == 1) info = gesv_mixed_gmres(A, piv, B, X, iter, c.opts);
            else {
                HermitianMatrix<T> H(Uplo::Lower, A);
                info = variant == 2 ? posv_mixed(H, B, X, iter, c.opts) : posv_mixed_gmres(H, B, X, iter, c.opts);
            }
        });
        r.flops = variant >= 2 ? potrf_fl<T>(c.n) : getrf_fl<T>(c.n);
        r.note = "iter=" + std::to_string(iter);
        if (info) { r.error = INFINITY; return r; }
        if (c.P.check) r.error = c.solve_resid(A0, X, B);
        return r;
    }
}

template <typename T>
Result r_posv(Case<T>& c, bool factor_only) {
    auto Ag = c.mat(c.n, c.n, "spd"), B = c.mat(c.n, c.P.nrhs);
    auto A0 = c.copy_of(Ag), B0 = c.copy_of(B);
    HermitianMatrix<T> A(Uplo::Lower, Ag);
    Result r;
    int64_t info = 0;
    r.time = c.timed([&] { info = factor_only ? potrf(A, c.opts) : posv(A, B, c.opts); });
    r.flops = potrf_fl<T>(c.n);
    if (info) { r.error = INFINITY; r.note = "info=" + std::to_string(info); return r; }
    if (c.P.check) {
        if (factor_only) potrs(A, B, c.opts);
        r.error = c.solve_resid(A0, B, B0);   // "spd" is generated as a full Hermitian matrix
    }
    return r;
}

template <typename T>
Result r_getri(Case<T>& c) {
    auto A = c.mat(c.n, c.n, "rands+n");
    auto A0 = c.copy_of(A);
    Result r;
    int64_t info = 0;
    r.time = c.timed([&] {
        Pivots piv;
        info = getrf(A, piv, c.opts);
        if (!info) info = getri(A, piv, c.opts);
    });
    r.flops = getrf_fl<T>(c.n) + cfac<T>() * 4.0 / 3 * double(c.n) * c.n * c.n;
    if (info) { r.error = INFINITY; return r; }
    if (c.P.check) {
        auto I = c.zeros(c.n, c.n);
        set(T(0), T(1), I, c.opts);
        gemm(T(1), A0, A, T(-1), I, c.opts);
        r.error = c.nrm(I) / (double(c.n) * c.nrm(A0) * c.nrm(A));
    }
    return r;
}

template <typename T>
Result r_trtri(Case<T>& c) {
    auto Tg = c.mat(c.n, c.n, "rands+n");
    auto T0g = c.copy_of(Tg);
    TriangularMatrix<T> L(Uplo::Lower, Diag::NonUnit, Tg), L0(Uplo::Lower, Diag::NonUnit, T0g);
    Result r;
    int64_t info = 0;
    r.time = c.timed([&] { info = trtri(L, c.opts); });
    r.flops = cfac<T>() * double(c.n) * c.n * c.n / 3;
    if (info) { r.error = INFINITY; return r; }
    if (c.P.check) {
        // L0 * inv(L) = I, inv(L) materialized as a general lower matrix
        auto Li = c.zeros(c.n, c.n);
        BaseTrapezoidMatrix<T> Ls(Uplo::Lower, Tg, MatrixKind::Trapezoid), Ld(Uplo::Lower, Li, MatrixKind::Trapezoid);
        copy<T, T>(Ls, Ld, c.opts);
        trmm(Side::Left, T(1), L0, Li, c.opts);
        auto I = c.zeros(c.n, c.n);
        set(T(0), T(1), I, c.opts);
        add(T(-1), I, T(1), Li, c.opts);
        r.error = c.nrm(Li) / double(c.n);
    }
    return r;
}

template <typename T>
Result r_geqrf(Case<T>& c) {
    auto A = c.mat(c.m, c.n);
    auto A0 = c.copy_of(A);
    TriangularFactors<T> Tf;
    Result r;
    r.time = c.timed([&] { geqrf(A, Tf, c.opts); });
    double m = double(c.m), n = double(c.n);
    r.flops = cfac<T>() * (c.m >= c.n ? 2 * m * n * n - 2.0 / 3 * n * n * n : 2 * n * m * m - 2.0 / 3 * m * m * m);
    if (c.P.check) {
        // Q R with R = triu(A) (m x n), Q applied by unmqr
        auto QR = c.zeros(c.m, c.n);
        BaseTrapezoidMatrix<T> Rt(Uplo::Upper, A, MatrixKind::Trapezoid), Qt(Uplo::Upper, QR, MatrixKind::Trapezoid);
        copy<T, T>(Rt, Qt, c.opts);
        unmqr(Side::Left, Op::NoTrans, A, Tf, QR, c.opts);
        add(T(-1), A0, T(1), QR, c.opts);
        r.error = c.nrm(QR) / (double(c.m) * c.nrm(A0));
    }
    return r;
}

template <typename T>
Result r_gelqf(Case<T>& c) {
    auto A = c.mat(c.m, c.n);
    auto A0 = c.copy_of(A);
    TriangularFactors<T> Tf;
    Result r;
    r.time = c.timed([&] { gelqf(A, Tf, c.opts); });
    double m = double(c.m), n = double(c.n);
    r.flops = cfac<T>() * (c.n >= c.m ? 2 * n * m * m - 2.0 / 3 * m * m * m : 2 * m * n * n - 2.0 / 3 * n * n * n);
    if (c.P.check) {
        auto LQ = c.zeros(c.m, c.n);
        BaseTrapezoidMatrix<T> Lt(Uplo::Lower, A, MatrixKind::Trapezoid), Qt(Uplo::Lower, LQ, MatrixKind::Trapezoid);
        copy<T, T>(Lt, Qt, c.opts);
        unmlq(Side::Right, Op::NoTrans, A, Tf, LQ, c.opts);
        add(T(-1), A0, T(1), LQ, c.opts);
        r.error = c.nrm(LQ) / (double(c.n) * c.nrm(A0));
    }
    return r;
}

template <typename T>
Result r_gels(Case<T>& c) {
    auto A = c.mat(c.m, c.n), BX = c.mat(std::max(c.m, c.n), c.P.nrhs);
    auto A0 = c.copy_of(A), B0 = c.copy_of(BX);
    TriangularFactors<T> Tf;
    Result r;
    r.time = c.timed([&] { gels(A, Tf, BX, c.opts); });
    r.flops = cfac<T>() * 2.0 * c.m * c.n * std::min(c.m, c.n);
    if (c.P.check) {
        Matrix<T> X = BX.slice(0, c.n - 1, 0, c.P.nrhs - 1);
        auto Rr = c.copy_of(B0.slice(0, c.m - 1, 0, c.P.nrhs - 1));
        gemm(T(-1), A0, X, T(1), Rr, c.opts);
        if (c.m >= c.n) {
            auto G = c.zeros(c.n, c.P.nrhs);
            gemm(T(1), conj_transpose(A0), Rr, T(0), G, c.opts);        // A^H (b - A x) = 0
            r.error = c.nrm(G) / (c.nrm(A0) * c.nrm(A0) * c.nrm(X) * double(c.n));
        } else {
            r.error = c.nrm(Rr) / (c.nrm(A0) * c.nrm(X) * double(c.n));
        }
    }
    return r;
}

template <typename T>
Result r_heev(Case<T>& c) {
    auto Ag = c.mat(c.n, c.n, "spd", 0.0);
    auto A0 = c.copy_of(Ag);
    HermitianMatrix<T> A(Uplo::Lower, Ag);
    auto Z = c.zeros(c.n, c.n);
    std::vector<R_<T>> L;
    Result r;
    r.time = c.timed([&] { heev(A, L, Z, c.opts); });
    r.flops = cfac<T>() * 4.0 / 3 * double(c.n) * c.n * c.n;
    if (c.P.check) {
        auto AZ = c.zeros(c.n, c.n), ZL = c.copy_of(Z);
        gemm(T(1), A0, Z, T(0), AZ, c.opts);
        std::vector<R_<T>> ones(c.n, R_<T>(1));
        scale_row_col(Equed::Col, ones, L, ZL, c.opts);
        add(T(-1), ZL, T(1), AZ, c.opts);
        r.error = c.nrm(AZ) / (double(c.n) * c.nrm(A0));
    }
    return r;
}

template <typename T>
Result r_svd(Case<T>& c) {
    auto A = c.mat(c.m, c.n);
    auto A0 = c.copy_of(A);
    int64_t k = std::min(c.m, c.n);
    auto U = c.zeros(c.m, k), VT = c.zeros(k, c.n);
    std::vector<R_<T>> S;
    Result r;
    r.time = c.timed([&] { svd(A, S, U, VT, c.opts); });
    r.flops = cfac<T>() * 8.0 / 3 * double(k) * k * k;
    if (c.P.check) {
        std::vector<R_<T>> ones(c.m, R_<T>(1));
        scale_row_col(Equed::Col, ones, S, U, c.opts);
        double a0 = c.nrm(A0);
        gemm(T(1), U, VT, T(-1), A0, c.opts);
        r.error = c.nrm(A0) / (double(k) * a0);
    }
    return r;
}

template <typename T>
Result r_hesv(Case<T>& c) {
    auto Ag = c.mat(c.n, c.n, "spd", 0.0), B = c.mat(c.n, c.P.nrhs);
    auto A0 = c.copy_of(Ag), B0 = c.copy_of(B);
    HermitianMatrix<T> A(Uplo::Lower, Ag);
    Result r;
    int64_t info = 0;
    r.time = c.timed([&] { std::vector<int64_t> ipiv; info = hesv(A, ipiv, B, c.opts); });
    r.flops = cfac<T>() * double(c.n) * c.n * c.n / 3;
    if (info) { r.error = INFINITY; return r; }
    if (c.P.check) r.error = c.solve_resid(A0, B, B0);
    return r;
}

template <typename T>
Result r_gbsv(Case<T>& c) {
    int64_t kl = std::max<int64_t>(1, c.nb / 4), ku = kl;
    auto Ag = c.mat(c.n, c.n, "rands+n"), B = c.mat(c.n, c.P.nrhs);
    auto A0g = c.copy_of(Ag), B0 = c.copy_of(B);
    BandMatrix<T> A(kl, ku, Ag), A0(kl, ku, A0g);
    Result r;
    int64_t info = 0;
    r.time = c.timed([&] { Pivots piv; info = gbsv(A, piv, B, c.opts); });
    if (info) { r.error = INFINITY; return r; }
    if (c.P.check) {
        auto Rm = c.copy_of(B0);
        gbmm(T(-1), A0, B, T(1), Rm, c.opts);
        r.error = c.nrm(Rm) / (double(c.n) * c.nrm(B0) * c.nrm(B));
    }
    return r;
}

template <typename T>
Result r_genorm(Case<T>& c) {
    auto A = c.mat(c.m, c.n);
    Result r;
    R_<T> v1 = 0;
    r.time = c.timed([&] { v1 = norm(Norm::One, A, c.opts); });
    r.flops = double(c.m) * c.n;
    if (c.P.check) {
        // one-norm of A == inf-norm of A^H (materialized)
        auto AH = c.zeros(c.n, c.m);
        copy<T, T>(conj_transpose(A), AH, c.opts);
        R_<T> v2 = norm(Norm::Inf, AH, c.opts);
        r.error = std::abs(double(v1 - v2)) / double(v1);
    }
    return r;
}


//------------------------------------------------------------------------------
// Breadth: the rest of the reference tester's routine list (test/test.cc:83-295)
template <typename T>
Result blas3_check(Case<T>& c, Matrix<T>& Cn, std::function<void(Matrix<T> const& X, Matrix<T>& Y)> expect,
                   double scale) {
    // C_new X == expect(X) for a random X
    auto X = c.mat(Cn.n(), 4), CX = c.zeros(Cn.m(), 4), Y = c.zeros(Cn.m(), 4);
    gemm(T(1), Cn, X, T(0), CX, c.opts);
    expect(X, Y);
    add(T(-1), CX, T(1), Y, c.opts);
    return Result{NAN, c.nrm(Y) / (scale * c.nrm(X)), 0, false, ""};
}

template <typename T>
Matrix<T> full_of(Case<T>& c, BaseTrapezoidMatrix<T> const& S, bool herm) {
    // dense copy of a Hermitian / symmetric matrix stored in one triangle
    auto F = c.zeros(S.n(), S.n());
    Matrix<T> G(S);
    G.set_uplo(Uplo::General);
    copy<T, T>(herm ? conj_transpose(G) : transpose(G), F, c.opts);
    BaseTrapezoidMatrix<T> Fs(S.uplo(), F, MatrixKind::Trapezoid), Gs(S.uplo(), G, MatrixKind::Trapezoid);
    copy<T, T>(Gs, Fs, c.opts);
    return F;
}

template <typename T>
Result r_rankk(Case<T>& c, int kind) {   // 0 syrk, 1 her2k, 2 syr2k
    auto A = c.mat(c.n, c.k), B = c.mat(c.n, c.k), Cg = c.mat(c.n, c.n, "spd", 0.0);
    auto C0 = c.copy_of(Cg);
    const bool herm = kind == 1;
    T alpha(1.5), beta(0.5);
    Result r;
    if (kind == 0) { SymmetricMatrix<T> C(Uplo::Lower, Cg); r.time = c.timed([&] { syrk(alpha, A, beta, C, c.opts); }); }
    else if (kind == 1) { HermitianMatrix<T> C(Uplo::Lower, Cg); r.time = c.timed([&] { her2k(alpha, A, B, R_<T>(0.5), C, c.opts); }); }
    else { SymmetricMatrix<T> C(Uplo::Lower, Cg); r.time = c.timed([&] { syr2k(alpha, A, B, beta, C, c.opts); }); }
    r.flops = cfac<T>() * double(c.k) * c.n * (c.n + 1) * (kind == 0 ? 1 : 2);
    if (c.P.check) {
        BaseTrapezoidMatrix<T> Cs(Uplo::Lower, Cg, MatrixKind::Trapezoid), C0s(Uplo::Lower, C0, MatrixKind::Trapezoid);
        auto Cn = full_of(c, Cs, herm), Cz = full_of(c, C0s, herm);
        auto res = blas3_check<T>(c, Cn, [&](Matrix<T> const& X, Matrix<T>& Y) {
            auto AX = c.zeros(c.k, 4), BX = c.zeros(c.k, 4);
            auto opA = herm ? conj_transpose(A) : transpose(A);
            auto opB = herm ? conj_transpose(B) : transpose(B);
            gemm(beta, Cz, X, T(0), Y, c.opts);
            if (kind == 0) { gemm(T(1), opA, X, T(0), AX, c.opts); gemm(alpha, A, AX, T(1), Y, c.opts); }
            else {
                gemm(T(1), opB, X, T(0), BX, c.opts); gemm(alpha, A, BX, T(1), Y, c.opts);
                gemm(T(1), opA, X, T(0), AX, c.opts); gemm(herm ? slate::conj(alpha) : alpha, B, AX, T(1), Y, c.opts);
            }
        }, c.nrm(A) * c.nrm(B) * 3 + c.nrm(C0));
        r.error = res.error;
    }
    return r;
}

template <typename T>
Result r_symm(Case<T>& c) {
    auto Ag = c.mat(c.m, c.m), B = c.mat(c.m, c.n), C = c.mat(c.m, c.n);
    auto C0 = c.copy_of(C);
    SymmetricMatrix<T> A(Uplo::Lower, Ag);
    T alpha(1), beta(0.5);
    Result r;
    r.time = c.timed([&] { symm(Side::Left, alpha, A, B, beta, C, c.opts); });
    r.flops = gemm_fl<T>(c.m, c.n, c.m);
    if (c.P.check) {
        BaseTrapezoidMatrix<T> As(Uplo::Lower, Ag, MatrixKind::Trapezoid);
        auto F = full_of(c, As, false);
        auto res = blas3_check<T>(c, C, [&](Matrix<T> const& X, Matrix<T>& Y) {
            auto BX = c.zeros(c.m, 4);
            gemm(T(1), B, X, T(0), BX, c.opts);
            gemm(beta, C0, X, T(0), Y, c.opts);
            gemm(alpha, F, BX, T(1), Y, c.opts);
        }, c.nrm(F) * c.nrm(B) + c.nrm(C0));
        r.error = res.error;
    }
    return r;
}

template <typename T>
Result r_gemm_m(Case<T>& c, int64_t method) {
    Options o = c.opts;
    o[Option::MethodGemm] = method;
    auto A = c.mat(c.m, c.k), B = c.mat(c.k, c.n), C = c.mat(c.m, c.n);
    auto C0 = c.copy_of(C);
    Result r;
    r.time = c.timed([&] { gemm(T(1), A, B, T(-1), C, o); });
    r.flops = gemm_fl<T>(c.m, c.n, c.k);
    if (c.P.check) {
        auto res = blas3_check<T>(c, C, [&](Matrix<T> const& X, Matrix<T>& Y) {
            auto BX = c.zeros(c.k, 4);
            gemm(T(1), B, X, T(0), BX, c.opts);
            gemm(T(-1), C0, X, T(0), Y, c.opts);
            gemm(T(1), A, BX, T(1), Y, c.opts);
        }, c.nrm(A) * c.nrm(B) + c.nrm(C0));
        r.error = res.error;
    }
    return r;
}

template <typename T>
Result r_getrs(Case<T>& c) {
    auto A = c.mat(c.n, c.n, "rands", -1, true), B = c.mat(c.n, c.P.nrhs);
    auto A0 = c.copy_of(A), B0 = c.copy_of(B);
    Pivots piv;
    int64_t info = getrf(A, piv, c.opts);
    Result r;
    if (info) { r.error = INFINITY; return r; }
    r.time = c.timed([&] { getrs(A, piv, B, c.opts); });
    r.flops = cfac<T>() * 2.0 * c.n * c.n * c.P.nrhs;
    if (c.P.check) r.error = c.solve_resid(A0, B, B0);
    return r;
}

template <typename T>
Result r_potrs(Case<T>& c, int variant) {   // 0 potrs, 1 potri
    auto Ag = c.mat(c.n, c.n, "spd"), B = c.mat(c.n, c.P.nrhs);
    auto A0 = c.copy_of(Ag), B0 = c.copy_of(B);
    HermitianMatrix<T> A(Uplo::Lower, Ag);
    Result r;
    if (potrf(A, c.opts)) { r.error = INFINITY; return r; }
    if (variant == 0) {
        r.time = c.timed([&] { potrs(A, B, c.opts); });
        r.flops = cfac<T>() * 2.0 * c.n * c.n * c.P.nrhs;
        if (c.P.check) r.error = c.solve_resid(A0, B, B0);
    } else {
        int64_t info = 0;
        r.time = c.timed([&] { info = potri(A, c.opts); });
        r.flops = cfac<T>() * 2.0 / 3 * double(c.n) * c.n * c.n;
        if (info) { r.error = INFINITY; return r; }
        if (c.P.check) {
            BaseTrapezoidMatrix<T> As(Uplo::Lower, Ag, MatrixKind::Trapezoid);
            auto Ai = full_of(c, As, true);
            auto I = c.zeros(c.n, c.n);
            set(T(0), T(1), I, c.opts);
            gemm(T(1), A0, Ai, T(-1), I, c.opts);
            r.error = c.nrm(I) / (double(c.n) * c.nrm(A0) * c.nrm(Ai));
        }
    }
    return r;
}

template <typename T>
Result r_gesv_v(Case<T>& c, int variant) {   // 0 nopiv, 1 tntpiv, 2 rbt
    if (variant == 0)
        return solve_case<T>(c, "rands+n", [&](Matrix<T>& A, Matrix<T>& B) { return gesv_nopiv(A, B, c.opts); },
                             getrf_fl<T>(c.n));
    if (variant == 1) {
        Options o = c.opts;
        o[Option::MethodLU] = int64_t(MethodLU::CALU);
        return solve_case<T>(c, "rands", [&, o](Matrix<T>& A, Matrix<T>& B) { Pivots piv; return gesv(A, piv, B, o); },
                             getrf_fl<T>(c.n));
    }
    auto A = c.mat(c.n, c.n, "rands", -1, true), B = c.mat(c.n, c.P.nrhs);
    auto A0 = c.copy_of(A), X = c.zeros(c.n, c.P.nrhs);
    Result r;
    int iter = 0;
    int64_t info = 0;
    r.time = c.timed([&] { info = gesv_rbt(A, B, X, iter, c.opts); });
    r.flops = getrf_fl<T>(c.n);
    r.note = "iter=" + std::to_string(iter);
    if (info) { r.error = INFINITY; return r; }
    if (c.P.check) r.error = c.solve_resid(A0, X, B);
    return r;
}

template <typename T>
Result r_condest(Case<T>& c, int variant) {   // 0 gecondest, 1 pocondest, 2 trcondest
    Result r;
    auto A = c.mat(c.n, c.n, variant == 1 ? "spd" : "rands+n");
    const double anorm = c.nrm(A);
    R_<T> rc = 0;
    if (variant == 0) {
        Pivots piv;
        getrf(A, piv, c.opts);
        r.time = c.timed([&] { rc = gecondest(Norm::One, A, R_<T>(anorm), c.opts); });
    } else if (variant == 1) {
        HermitianMatrix<T> H(Uplo::Lower, A);
        potrf(H, c.opts);
        r.time = c.timed([&] { rc = pocondest(Norm::One, H, R_<T>(anorm), c.opts); });
    } else {
        TriangularMatrix<T> L(Uplo::Lower, Diag::NonUnit, A);
        r.time = c.timed([&] { rc = trcondest(Norm::One, L, c.opts); });
    }
    r.flops = cfac<T>() * 4.0 * c.n * c.n;
    r.error = (rc > 0 && rc <= 1) ? 0.0 : INFINITY;   // an estimate: only its range is checked
    char b[48];
    std::snprintf(b, sizeof(b), "rcond=%.3e", double(rc));
    r.note = b;
    return r;
}

template <typename T>
Result r_unmqr(Case<T>& c, bool lq) {
    auto A = c.mat(c.m, c.n), C = c.mat(lq ? c.n : c.m, c.P.nrhs);
    auto C0 = c.copy_of(C);
    TriangularFactors<T> Tf;
    if (lq) gelqf(A, Tf, c.opts); else geqrf(A, Tf, c.opts);
    Result r;
    r.time = c.timed([&] {
        if (lq) unmlq(Side::Left, Op::ConjTrans, A, Tf, C, c.opts);
        else unmqr(Side::Left, Op::ConjTrans, A, Tf, C, c.opts);
    });
    r.flops = cfac<T>() * 4.0 * c.m * c.n * c.P.nrhs;
    if (c.P.check) {   // Q (Q^H C) = C
        if (lq) unmlq(Side::Left, Op::NoTrans, A, Tf, C, c.opts);
        else unmqr(Side::Left, Op::NoTrans, A, Tf, C, c.opts);
        add(T(-1), C0, T(1), C, c.opts);
        r.error = c.nrm(C) / (c.nrm(C0) * double(c.m));
    }
    return r;
}

template <typename T>
Result r_cholqr(Case<T>& c) {
    if (c.m < c.n) { Result r; r.skipped = true; r.note = "m >= n"; return r; }
    auto A = c.mat(c.m, c.n);
    auto A0 = c.copy_of(A), Rm = c.zeros(c.n, c.n);
    Result r;
    int64_t info = 0;
    r.time = c.timed([&] { info = cholqr(A, Rm, c.opts); });
    r.flops = cfac<T>() * (2.0 * c.m * c.n * c.n + double(c.n) * c.n * c.n / 3);
    if (info) { r.error = INFINITY; return r; }
    if (c.P.check) {   // Q R = A0
        TriangularMatrix<T> Rt(Uplo::Upper, Diag::NonUnit, Rm);
        auto QR = c.copy_of(A);
        trmm(Side::Right, T(1), Rt, QR, c.opts);
        add(T(-1), A0, T(1), QR, c.opts);
        r.error = c.nrm(QR) / (double(c.m) * c.nrm(A0));
    }
    return r;
}

template <typename T>
Result r_band(Case<T>& c, int variant) {   // 0 gbtrf+gbtrs, 1 pbsv, 2 pbtrf+pbtrs, 3 gbmm, 4 hbmm, 5 tbsm, 6 gbtrs, 7 pbtrs, 8 tbsm with pivots
    const int64_t kd = std::max<int64_t>(1, c.nb / 2);
    Result r;
    if (variant == 1 || variant == 2 || variant == 4 || variant == 7) {
        auto Ag = c.mat(c.n, c.n, "rands", -1, true), B = c.mat(c.n, c.P.nrhs);
        // Hermitian band with a dominant diagonal: H = band(A + A^H) + 4 kd I
        auto F = c.zeros(c.n, c.n);
        copy<T, T>(conj_transpose(Ag), F, c.opts);
        add(T(1), Ag, T(1), F, c.opts);
        BandMatrix<T> Fb(kd, kd, F);
        auto D = c.zeros(c.n, c.n);
        set(T(0), T(4 * kd + 4), D, c.opts);
        add(T(1), D, T(1), F, c.opts);
        auto Fz = c.zeros(c.n, c.n);   // dense band copy for the residual
        {
            auto Tmp = c.copy_of(F);
            BandMatrix<T> Tb(kd, kd, Tmp);
            auto I = c.zeros(c.n, c.n);
            set(T(0), T(1), I, c.opts);
            gbmm(T(1), Tb, I, T(0), Fz, c.opts);
        }
        auto B0 = c.copy_of(B);
        HermitianBandMatrix<T> H(Uplo::Lower, kd, F);
        if (variant == 4) {
            auto C = c.zeros(c.n, c.P.nrhs);
            r.time = c.timed([&] { hbmm(Side::Left, T(1), H, B, T(0), C, c.opts); });
            r.flops = cfac<T>() * 2.0 * c.n * (2 * kd + 1) * c.P.nrhs;
            if (c.P.check) {
                gemm(T(-1), Fz, B, T(1), C, c.opts);
                r.error = c.nrm(C) / (c.nrm(Fz) * c.nrm(B) * double(c.n));
            }
            return r;
        }
        int64_t info = 0;
        if (variant == 7) {
            info = pbtrf(H, c.opts);
            if (info) { r.error = INFINITY; return r; }
            r.time = c.timed([&] { pbtrs(H, B, c.opts); });
            r.flops = cfac<T>() * 4.0 * c.n * kd * c.P.nrhs;
            if (c.P.check) r.error = c.solve_resid(Fz, B, B0);
            return r;
        }
        r.time = c.timed([&] {
            if (variant == 1) info = pbsv(H, B, c.opts);
            else { info = pbtrf(H, c.opts); if (!info) pbtrs(H, B, c.opts); }
        });
        r.flops = cfac<T>() * double(c.n) * kd * kd;
        if (info) { r.error = INFINITY; return r; }
        if (c.P.check) r.error = c.solve_resid(Fz, B, B0);
        return r;
    }
    auto Ag = c.mat(c.n, c.n, "rands+n", -1, true), B = c.mat(c.n, c.P.nrhs);
    auto A0g = c.copy_of(Ag), B0 = c.copy_of(B);
    BandMatrix<T> A(kd, kd / 2 + 1, Ag), A0(kd, kd / 2 + 1, A0g);
    if (variant == 3) {
        auto C = c.zeros(c.n, c.P.nrhs);
        r.time = c.timed([&] { gbmm(T(1), A0, B, T(0), C, c.opts); });
        r.flops = cfac<T>() * 2.0 * c.n * (1.5 * kd + 2) * c.P.nrhs;
        if (c.P.check) {   // (A0 B) X via the band multiply twice
            auto C2 = c.zeros(c.n, c.P.nrhs);
            gbmm(T(1), A0, B, T(0), C2, c.opts);
            add(T(-1), C, T(1), C2, c.opts);
            r.error = c.nrm(C2) / std::max(1e-300, c.nrm(C));
        }
        return r;
    }
    if (variant == 5) {
        TriangularBandMatrix<T> L(Uplo::Lower, Diag::NonUnit, kd, Ag);
        auto X = c.copy_of(B);
        r.time = c.timed([&] { tbsm(Side::Left, T(1), L, X, c.opts); });
        r.flops = cfac<T>() * double(c.n) * kd * c.P.nrhs;
        if (c.P.check) {   // L X == B through the dense triangle of the band
            auto D = c.zeros(c.n, c.n);
            BaseTrapezoidMatrix<T> Ls(Uplo::Lower, A0g, MatrixKind::Trapezoid), Ds(Uplo::Lower, D, MatrixKind::Trapezoid);
            copy<T, T>(Ls, Ds, c.opts);
            BandMatrix<T> Db(kd, 0, D);
            auto LX = c.zeros(c.n, c.P.nrhs);
            gbmm(T(1), Db, X, T(0), LX, c.opts);
            add(T(-1), B0, T(1), LX, c.opts);
            r.error = c.nrm(LX) / (c.nrm(B0) * double(c.n));
        }
        return r;
    }
    if (variant == 8) {   // tbsm with row interchanges (reference src/tbsmPivots.cc)
        scale(R_<T>(1), R_<T>(2 * kd), Ag, c.opts);   // |L(i, j)| <= 1 / (4 kd): no growth in the sweep
        TriangularBandMatrix<T> L(Uplo::Lower, Diag::Unit, kd, Ag);
        const int64_t mt = Ag.mt();
        std::vector<int64_t> r0(mt + 1, 0);
        for (int64_t k = 0; k < mt; ++k) r0[k + 1] = r0[k] + Ag.tileMb(k);
        // pivots of tile k: rows within the band reach, as gbtrf produces them
        Pivots piv(mt);
        uint64_t s = 7;
        for (int64_t k = 0; k < mt; ++k)
            for (int64_t row = r0[k]; row < r0[k + 1]; ++row) {
                s = s * 6364136223846793005ull + 1442695040888963407ull;
                const int64_t p = row + int64_t((s >> 33) % uint64_t(std::min(c.n, row + kd + 1) - row));
                const int64_t tp = std::upper_bound(r0.begin(), r0.end(), p) - r0.begin() - 1;
                piv[k].emplace_back(tp - k, p - r0[tp]);
            }
        auto X = c.copy_of(B);
        r.time = c.timed([&] { tbsm(Side::Left, T(1), L, piv, X, c.opts); });
        r.flops = cfac<T>() * double(c.n) * kd * c.P.nrhs;
        if (c.P.check) {   // the reference's sweep on the host: tile k's swaps, then its eliminations
            std::vector<T> l, xs, x1;
            gather(Ag, l, c.opts);
            gather(B, xs, c.opts);
            gather(X, x1, c.opts);
            const int64_t n = c.n, nr = c.P.nrhs;
            for (int64_t k = 0; k < mt; ++k) {
                for (int64_t t = 0; t < r0[k + 1] - r0[k]; ++t) {
                    const int64_t row = r0[k] + t, p = r0[k + piv[k][t].tileIndex()] + piv[k][t].elementOffset();
                    if (p != row)
                        for (int64_t j = 0; j < nr; ++j) std::swap(xs[size_t(row + j * n)], xs[size_t(p + j * n)]);
                }
                for (int64_t col = r0[k]; col < r0[k + 1]; ++col)
                    for (int64_t i = col + 1; i <= std::min(n - 1, col + kd); ++i)
                        for (int64_t j = 0; j < nr; ++j)
                            xs[size_t(i + j * n)] -= l[size_t(i + col * n)] * xs[size_t(col + j * n)];
            }
            double err = 0, mx = 1e-300;
            for (size_t i = 0; i < xs.size(); ++i) {
                err = std::max(err, double(std::abs(x1[i] - xs[i])));
                mx = std::max(mx, double(std::abs(xs[i])));
            }
            r.error = err / (mx * double(kd));
        }
        return r;
    }
    int64_t info = 0;
    if (variant == 6) {
        Pivots piv;
        info = gbtrf(A, piv, c.opts);
        if (info) { r.error = INFINITY; return r; }
        r.time = c.timed([&] { gbtrs(A, piv, B, c.opts); });
        r.flops = cfac<T>() * 2.0 * c.n * (2.5 * kd + 1) * c.P.nrhs;
    } else {
        r.time = c.timed([&] { Pivots piv; info = gbtrf(A, piv, c.opts); if (!info) gbtrs(A, piv, B, c.opts); });
    }
    if (variant != 6) r.flops = cfac<T>() * 2.0 * c.n * kd * (1.5 * kd + 1);
    if (info) { r.error = INFINITY; return r; }
    if (c.P.check) {
        auto Rm = c.copy_of(B0);
        gbmm(T(-1), A0, B, T(1), Rm, c.opts);
        r.error = c.nrm(Rm) / (double(c.n) * c.nrm(B0) * c.nrm(B));
    }
    return r;
}

template <typename T>
Result r_hetrf(Case<T>& c) {
    auto Ag = c.mat(c.n, c.n, "rands", -1, true), B = c.mat(c.n, c.P.nrhs);
    // indefinite Hermitian: A + A^H
    auto H0 = c.zeros(c.n, c.n);
    copy<T, T>(conj_transpose(Ag), H0, c.opts);
    add(T(1), Ag, T(1), H0, c.opts);
    auto Hg = c.copy_of(H0), B0 = c.copy_of(B);
    HermitianMatrix<T> H(Uplo::Lower, Hg);
    std::vector<int64_t> ipiv;
    Result r;
    int64_t info = 0;
    r.time = c.timed([&] { info = hetrf(H, ipiv, c.opts); });
    r.flops = cfac<T>() * double(c.n) * c.n * c.n / 3;
    if (info) { r.error = INFINITY; return r; }
    if (c.P.check) {
        hetrs(H, ipiv, B, c.opts);
        r.error = c.solve_resid(H0, B, B0);
    }
    return r;
}

template <typename T>
Result r_hesv_aasen(Case<T>& c) {
    auto Ag = c.mat(c.n, c.n, "rands", -1, true), B = c.mat(c.n, c.P.nrhs);
    auto H0 = c.zeros(c.n, c.n);
    copy<T, T>(conj_transpose(Ag), H0, c.opts);
    add(T(1), Ag, T(1), H0, c.opts);
    auto Hg = c.copy_of(H0), B0 = c.copy_of(B), Tg = c.zeros(c.n, c.n);
    HermitianMatrix<T> H(Uplo::Lower, Hg);
    BandMatrix<T> Tb(c.nb, c.nb, Tg);
    Matrix<T> W;
    Pivots p1, p2;
    Result r;
    int64_t info = 0;
    r.time = c.timed([&] { info = hesv(H, p1, Tb, p2, W, B, c.opts); });
    r.flops = cfac<T>() * double(c.n) * c.n * c.n / 3;
    if (info) { r.error = INFINITY; return r; }
    if (c.P.check) r.error = c.solve_resid(H0, B, B0);
    return r;
}

template <typename T>
Result r_vals(Case<T>& c, int variant) {   // 0 heev values, 1 svd values, 2 hegv
    Result r;
    if (variant == 1) {
        auto A = c.mat(c.m, c.n, "rands", -1, true);
        auto A0 = c.copy_of(A);
        std::vector<R_<T>> S;
        r.time = c.timed([&] { svd_vals(A, S, c.opts); });
        r.flops = cfac<T>() * 8.0 / 3 * double(std::min(c.m, c.n)) * c.m * c.n;
        // sum of squares of the singular values == ||A||_F^2
        double ss = 0;
        for (auto v : S) ss += double(v) * double(v);
        double f = double(norm(Norm::Fro, A0, c.opts));
        r.error = std::abs(ss - f * f) / (f * f * double(c.n));
        return r;
    }
    auto Ag = c.mat(c.n, c.n, "spd", 0.0);
    auto A0 = c.copy_of(Ag);
    HermitianMatrix<T> A(Uplo::Lower, Ag);
    std::vector<R_<T>> L;
    if (variant == 0) {
        Matrix<T> none;
        r.time = c.timed([&] { heev(A, L, none, c.opts); });
        r.flops = cfac<T>() * 4.0 / 3 * double(c.n) * c.n * c.n;
        if (c.P.check) {   // the values-only path against the vectors path
            auto Ag2 = c.copy_of(A0);
            HermitianMatrix<T> A2(Uplo::Lower, Ag2);
            auto Z = c.zeros(c.n, c.n);
            std::vector<R_<T>> L2;
            heev(A2, L2, Z, c.opts);
            double mx = 0;
            for (int64_t i = 0; i < c.n; ++i) mx = std::max(mx, std::abs(double(L[i]) - double(L2[i])));
            r.error = mx / (double(c.n) * c.nrm(A0));
        }
        return r;
    }
    auto Bg = c.mat(c.n, c.n, "spd");
    HermitianMatrix<T> B(Uplo::Lower, Bg);
    auto B0 = c.copy_of(Bg);
    auto Z = c.zeros(c.n, c.n);
    r.time = c.timed([&] { hegv(1, A, B, L, Z, c.opts); });
    r.flops = cfac<T>() * 3.0 * double(c.n) * c.n * c.n;
    if (c.P.check) {   // A Z = B Z Lambda
        auto AZ = c.zeros(c.n, c.n), BZ = c.zeros(c.n, c.n);
        gemm(T(1), A0, Z, T(0), AZ, c.opts);
        gemm(T(1), B0, Z, T(0), BZ, c.opts);
        std::vector<R_<T>> ones(c.n, R_<T>(1));
        scale_row_col(Equed::Col, ones, L, BZ, c.opts);
        add(T(-1), BZ, T(1), AZ, c.opts);
        r.error = c.nrm(AZ) / (double(c.n) * c.nrm(A0) * c.nrm(Z));
    }
    return r;
}

template <typename T>
Result r_tridiag(Case<T>& c, int variant) {   // 0 sterf, 1 steqr2, 2 stedc (via heev method dc on a tridiagonal)
    using R = R_<T>;
    const int64_t n = c.n;
    std::vector<R> d(n), e(std::max<int64_t>(n - 1, 0));
    for (int64_t i = 0; i < n; ++i) d[i] = R(2) + R(i % 7) / R(10);
    for (int64_t i = 0; i + 1 < n; ++i) e[i] = R(-1) + R(i % 5) / R(20);
    auto d0 = d;
    auto e0 = e;
    Result r;
    if (variant == 0) {
        r.time = c.timed([&] { sterf<R>(d, e, c.opts); });
        double s0 = 0, s1 = 0;
        for (auto v : d0) s0 += double(v);
        for (auto v : d) s1 += double(v);
        r.error = std::abs(s0 - s1) / (std::abs(s0) * double(n));   // trace preserved
        r.flops = 30.0 * n * n;
        return r;
    }
    auto Z = c.zeros(n, n);
    set(T(0), T(1), Z, c.opts);
    r.time = c.timed([&] { steqr2(Job::Vec, d, e, Z, c.opts); });
    r.flops = 6.0 * double(n) * n * n;
    if (c.P.check) {
        // T Z = Z diag(d) with T built as a dense tridiagonal
        auto Tm = c.zeros(n, n);
        std::function<T(int64_t, int64_t)> tv = [&](int64_t i, int64_t j) -> T {
            if (i == j) return T(d0[i]);
            if (i == j + 1) return T(e0[j]);
            if (j == i + 1) return T(e0[i]);
            return T(0);
        };
        set(tv, Tm, c.opts);
        auto TZ = c.zeros(n, n), ZL = c.copy_of(Z);
        gemm(T(1), Tm, Z, T(0), TZ, c.opts);
        std::vector<R> ones(n, R(1));
        scale_row_col(Equed::Col, ones, d, ZL, c.opts);
        add(T(-1), ZL, T(1), TZ, c.opts);
        r.error = c.nrm(TZ) / (double(n) * c.nrm(Tm));
    }
    return r;
}

template <typename T>
Result r_aux(Case<T>& c, int variant) {   // 0 add, 1 copy, 2 scale, 3 set, 4 trtrm, 5 colnorms, 6 henorm, 7 redistribute
    auto A = c.mat(c.m, c.n, "rands", -1, true), B = c.mat(c.m, c.n);
    auto A0 = c.copy_of(A), B0 = c.copy_of(B);
    Result r;
    r.flops = double(c.m) * c.n;
    switch (variant) {
        case 0:
            r.time = c.timed([&] { add(T(2), A, T(-1), B, c.opts); });
            if (c.P.check) { add(T(-2), A0, T(1), B, c.opts); add(T(1), B0, T(1), B, c.opts); r.error = c.nrm(B) / c.nrm(B0); }
            break;
        case 1:
            r.time = c.timed([&] { copy<T, T>(A, B, c.opts); });
            if (c.P.check) { add(T(-1), A0, T(1), B, c.opts); r.error = c.nrm(B); }
            break;
        case 2:
            r.time = c.timed([&] { scale(R_<T>(3), R_<T>(2), A, c.opts); });
            if (c.P.check) { add(T(-1.5), A0, T(1), A, c.opts); r.error = c.nrm(A) / c.nrm(A0); }
            break;
        case 3:
            r.time = c.timed([&] { set(T(0.5), T(2), A, c.opts); });
            if (c.P.check) {
                double e = double(norm(Norm::Max, A, c.opts));
                r.error = std::abs(e - 2.0) / 2.0;
            }
            break;
        case 4: {
            if (c.m != c.n) { r.skipped = true; r.note = "square only"; break; }
            TriangularMatrix<T> L(Uplo::Lower, Diag::NonUnit, A);
            r.time = c.timed([&] { trtrm(L, c.opts); });
            r.flops = cfac<T>() * double(c.n) * c.n * c.n / 3;
            if (c.P.check) {   // L^H L from the original lower triangle
                auto Lg = c.zeros(c.n, c.n);
                BaseTrapezoidMatrix<T> Ls(Uplo::Lower, A0, MatrixKind::Trapezoid), Ld(Uplo::Lower, Lg, MatrixKind::Trapezoid);
                copy<T, T>(Ls, Ld, c.opts);
                auto P = c.zeros(c.n, c.n);
                gemm(T(1), conj_transpose(Lg), Lg, T(0), P, c.opts);
                BaseTrapezoidMatrix<T> Rs(Uplo::Lower, A, MatrixKind::Trapezoid), Ps(Uplo::Lower, P, MatrixKind::Trapezoid);
                add(T(-1), Rs, T(1), Ps, c.opts);
                r.error = double(norm(Norm::Max, Ps, c.opts)) / (c.nrm(Lg) * c.nrm(Lg));
            }
            break;
        }
        case 5: {
            std::vector<R_<T>> v(c.n);
            r.time = c.timed([&] { colNorms(Norm::Max, A, v.data(), c.opts); });
            if (c.P.check) {
                double mx = 0;
                for (auto x : v) mx = std::max(mx, double(x));
                const double am = double(norm(Norm::Max, A, c.opts));
                r.error = std::abs(mx - am) / am;   // max over the column maxima == max norm
            }
            break;
        }
        case 6: {
            if (c.m != c.n) { r.skipped = true; r.note = "square only"; break; }
            HermitianMatrix<T> H(Uplo::Lower, A);
            R_<T> v1 = 0;
            r.time = c.timed([&] { v1 = norm(Norm::One, H, c.opts); });
            if (c.P.check) {
                BaseTrapezoidMatrix<T> Hs(Uplo::Lower, A, MatrixKind::Trapezoid);
                auto F = full_of(c, Hs, true);
                // the Hermitian matrix the stored triangle stands for has a
                // real diagonal (LAPACK lanhe reads only its real part):
                // F = (F + F^H) / 2 keeps the off-diagonal, drops Im(diag)
                auto Ft = c.zeros(c.n, c.n);
                copy<T, T>(conj_transpose(F), Ft, c.opts);
                add(T(0.5), Ft, T(0.5), F, c.opts);
                r.error = std::abs(double(v1) - c.nrm(F)) / c.nrm(F);
            }
            break;
        }
        case 7: {
            // 2D block-cyclic -> transposed-grid layout with another tile size and back
            auto g = default_grid();
            Matrix<T> Bt(c.m, c.n, std::max<int64_t>(1, c.nb / 2 + 3), g->transposed());
            Bt.insertLocalTiles(c.P.target);
            r.time = c.timed([&] { redistribute(A, Bt, c.opts); });
            if (c.P.check) {
                auto Back = c.zeros(c.m, c.n);
                redistribute(Bt, Back, c.opts);
                add(T(-1), A0, T(1), Back, c.opts);
                r.error = c.nrm(Back) / c.nrm(A0);
            }
            break;
        }
        default: break;
    }
    return r;
}

//------------------------------------------------------------------------------
// Breadth 2: stage-level eigen / SVD routines, the remaining solve variants,
// band / symmetric / triangular norms, trapezoid aux variants, sy* solvers.

/// dense copy of a Hermitian band (lower, kd) through hbmm with the identity
template <typename T>
Matrix<T> dense_hband(Case<T>& c, HermitianBandMatrix<T> const& H) {
    auto I = c.zeros(H.n(), H.n()), F = c.zeros(H.n(), H.n());
    set(T(0), T(1), I, c.opts);
    hbmm(Side::Left, T(1), H, I, T(0), F, c.opts);
    return F;
}

/// dense copy of a general band through gbmm with the identity
template <typename T>
Matrix<T> dense_band(Case<T>& c, BandMatrix<T> const& B) {
    auto I = c.zeros(B.n(), B.n()), F = c.zeros(B.m(), B.n());
    set(T(0), T(1), I, c.opts);
    gbmm(T(1), B, I, T(0), F, c.opts);
    return F;
}

/// Hermitian test matrix (A + A^H) / 2 from the main operand
template <typename T>
Matrix<T> herm_of(Case<T>& c, int64_t n) {
    auto Ag = c.mat(n, n, "rands", -1, true);
    auto H = c.zeros(n, n);
    copy<T, T>(conj_transpose(Ag), H, c.opts);
    add(T(0.5), Ag, T(0.5), H, c.opts);
    return H;
}

template <typename T>
Result r_he2hb(Case<T>& c, int variant) {   // 0 he2hb (A = Q B Q^H), 1 unmtr_he2hb (Q (Q^H C) = C)
    auto A = herm_of(c, c.n);
    auto A0 = c.copy_of(A);
    std::vector<TriangularFactors<T>> Ts;
    Result r;
    const double n = double(c.n);
    if (variant == 0) {
        r.time = c.timed([&] { he2hb(A, Ts, c.opts); });
        r.flops = cfac<T>() * 4.0 / 3 * n * n * n;
        if (c.P.check) {
            HermitianBandMatrix<T> Hb(Uplo::Lower, c.nb, A);
            auto F = dense_hband(c, Hb);
            unmtr_he2hb(Side::Left, Op::NoTrans, A, Ts, F, c.opts);
            unmtr_he2hb(Side::Right, Op::ConjTrans, A, Ts, F, c.opts);
            add(T(-1), A0, T(1), F, c.opts);
            r.error = c.nrm(F) / (n * c.nrm(A0));
        }
        return r;
    }
    he2hb(A, Ts, c.opts);
    auto C = c.mat(c.n, c.P.nrhs);
    auto C0 = c.copy_of(C);
    r.time = c.timed([&] { unmtr_he2hb(Side::Left, Op::ConjTrans, A, Ts, C, c.opts); });
    r.flops = cfac<T>() * 2.0 * n * n * c.P.nrhs;
    if (c.P.check) {
        unmtr_he2hb(Side::Left, Op::NoTrans, A, Ts, C, c.opts);
        add(T(-1), C0, T(1), C, c.opts);
        r.error = c.nrm(C) / (n * c.nrm(C0));
    }
    return r;
}

template <typename T>
Result r_hb2st(Case<T>& c, int variant) {   // 0 hb2st (Frobenius norm preserved), 1 unmtr_hb2st
    using R = R_<T>;
    auto A = herm_of(c, c.n);
    const int64_t kd = std::max<int64_t>(1, c.nb / 2);
    HermitianBandMatrix<T> Hb(Uplo::Lower, kd, A);
    std::vector<R> d, e;
    BandReflectors<T> V;
    Result r;
    const double n = double(c.n);
    if (variant == 0) {
        r.time = c.timed([&] { hb2st(Hb, d, e, V, c.opts); });
        r.flops = cfac<T>() * 6.0 * n * n * kd;
        if (c.P.check) {
            // orthogonal similarity: ||band||_F^2 = sum d^2 + 2 sum e^2
            const double f = double(norm(Norm::Fro, dense_hband(c, Hb), c.opts));
            double t = 0;
            for (auto v : d) t += double(v) * double(v);
            for (auto v : e) t += 2.0 * double(v) * double(v);
            r.error = std::abs(t - f * f) / (f * f * n);
        }
        return r;
    }
    hb2st(Hb, d, e, V, c.opts);
    auto C = c.mat(c.n, c.P.nrhs);
    auto C0 = c.copy_of(C);
    r.time = c.timed([&] { unmtr_hb2st(Side::Left, Op::NoTrans, V, C, c.opts); });
    r.flops = cfac<T>() * 2.0 * n * n * c.P.nrhs;
    if (c.P.check) {
        unmtr_hb2st(Side::Left, Op::ConjTrans, V, C, c.opts);
        add(T(-1), C0, T(1), C, c.opts);
        r.error = c.nrm(C) / (n * c.nrm(C0));
    }
    return r;
}

template <typename T>
Result r_ge2tb(Case<T>& c) {   // A = U B V^H with B upper band of width nb
    if (c.m < c.n) { Result r; r.skipped = true; r.note = "m >= n"; return r; }
    auto A = c.mat(c.m, c.n, "rands", -1, true);
    auto A0 = c.copy_of(A);
    std::vector<TriangularFactors<T>> TU, TV;
    Result r;
    r.time = c.timed([&] { ge2tb(A, TU, TV, c.opts); });
    r.flops = cfac<T>() * 4.0 * double(c.n) * c.n * (c.m - c.n / 3.0);
    if (c.P.check) {
        BandMatrix<T> Bb(0, c.nb, A);
        auto F = dense_band(c, Bb);
        unmbr_ge2tb(Side::Left, Op::NoTrans, A, TU, F, c.opts);
        unmbr_ge2tb(Side::Right, Op::NoTrans, A, TV, F, c.opts);
        add(T(-1), A0, T(1), F, c.opts);
        r.error = c.nrm(F) / (double(c.m) * c.nrm(A0));
    }
    return r;
}

template <typename T>
Result r_tb2bd(Case<T>& c, int variant) {   // 0 tb2bd (Frobenius preserved), 1 unmbr_tb2bd
    using R = R_<T>;
    auto A = c.mat(c.n, c.n, "rands", -1, true);
    const int64_t kd = std::max<int64_t>(1, c.nb / 2);
    TriangularBandMatrix<T> Tb(Uplo::Upper, Diag::NonUnit, kd, A);
    std::vector<R> d, e;
    BandReflectors<T> U, V;
    Result r;
    const double n = double(c.n);
    if (variant == 0) {
        r.time = c.timed([&] { tb2bd(Tb, d, e, U, V, c.opts); });
        r.flops = cfac<T>() * 8.0 * n * n * kd;
        if (c.P.check) {
            BandMatrix<T> Bb(0, kd, A);
            const double f = double(norm(Norm::Fro, dense_band(c, Bb), c.opts));
            double t = 0;
            for (auto v : d) t += double(v) * double(v);
            for (auto v : e) t += double(v) * double(v);
            r.error = std::abs(t - f * f) / (f * f * n);
        }
        return r;
    }
    tb2bd(Tb, d, e, U, V, c.opts);
    auto C = c.mat(c.n, c.P.nrhs);
    auto C0 = c.copy_of(C);
    r.time = c.timed([&] { unmbr_tb2bd(Side::Left, Op::NoTrans, U, C, c.opts); });
    r.flops = cfac<T>() * 2.0 * n * n * c.P.nrhs;
    if (c.P.check) {
        unmbr_tb2bd(Side::Left, Op::ConjTrans, U, C, c.opts);
        add(T(-1), C0, T(1), C, c.opts);
        r.error = c.nrm(C) / (n * c.nrm(C0));
    }
    return r;
}

/// the test tridiagonal / bidiagonal of the stage tests
template <typename R>
void test_tridiag(int64_t n, std::vector<R>& d, std::vector<R>& e) {
    d.resize(n);
    e.assign(std::max<int64_t>(n - 1, 0), R(0));
    for (int64_t i = 0; i < n; ++i) d[i] = R(2) + R(i % 7) / R(10);
    for (int64_t i = 0; i + 1 < n; ++i) e[i] = R(-1) + R(i % 5) / R(20);
}

template <typename T>
Result r_bdsqr(Case<T>& c) {   // B = U diag(s) VT for an upper bidiagonal B
    using R = R_<T>;
    const int64_t n = c.n;
    std::vector<R> d, e;
    test_tridiag(n, d, e);
    auto d0 = d;
    auto e0 = e;
    auto U = c.zeros(n, n), VT = c.zeros(n, n);
    set(T(0), T(1), U, c.opts);
    set(T(0), T(1), VT, c.opts);
    Result r;
    r.time = c.timed([&] { bdsqr(Job::Vec, Job::Vec, d, e, U, VT, c.opts); });
    r.flops = 12.0 * double(n) * n * n;
    if (c.P.check) {
        auto Bm = c.zeros(n, n);
        std::function<T(int64_t, int64_t)> bv = [&](int64_t i, int64_t j) -> T {
            if (i == j) return T(d0[i]);
            if (j == i + 1) return T(e0[i]);
            return T(0);
        };
        set(bv, Bm, c.opts);
        std::vector<R> ones(n, R(1));
        auto US = c.copy_of(U);
        scale_row_col(Equed::Col, ones, d, US, c.opts);
        gemm(T(1), US, VT, T(-1), Bm, c.opts);
        r.error = c.nrm(Bm) / (double(n) * 4.0);
    }
    return r;
}

template <typename T>
Result r_stedc(Case<T>& c) {   // T Q = Q diag(lambda), Q distributed
    using R = R_<T>;
    if constexpr (is_complex_v<T>) {
        Result r; r.skipped = true; r.note = "real types (stedc works on R)"; return r;
    } else {
        const int64_t n = c.n;
        std::vector<R> d, e;
        test_tridiag(n, d, e);
        auto d0 = d;
        auto e0 = e;
        auto Q = c.zeros(n, n);
        Result r;
        r.time = c.timed([&] { stedc(d, e, Q, c.opts); });
        r.flops = 4.0 / 3 * double(n) * n * n;
        if (c.P.check) {
            auto Tm = c.zeros(n, n);
            std::function<T(int64_t, int64_t)> tv = [&](int64_t i, int64_t j) -> T {
                if (i == j) return T(d0[i]);
                if (i == j + 1) return T(e0[j]);
                if (j == i + 1) return T(e0[i]);
                return T(0);
            };
            set(tv, Tm, c.opts);
            auto TQ = c.zeros(n, n), QL = c.copy_of(Q);
            gemm(T(1), Tm, Q, T(0), TQ, c.opts);
            std::vector<R> ones(n, R(1));
            scale_row_col(Equed::Col, ones, d, QL, c.opts);
            add(T(-1), QL, T(1), TQ, c.opts);
            r.error = c.nrm(TQ) / (double(n) * c.nrm(Tm));
        }
        return r;
    }
}

template <typename T>
Result r_hegst(Case<T>& c) {   // itype 1: C = L^{-1} A L^{-H}; check L C L^H = A
    auto A = herm_of(c, c.n);
    auto A0 = c.copy_of(A);
    auto Bg = c.mat(c.n, c.n, "spd");
    HermitianMatrix<T> Bh(Uplo::Lower, Bg);
    if (potrf(Bh, c.opts)) { Result r; r.error = INFINITY; return r; }
    HermitianMatrix<T> Ah(Uplo::Lower, A);
    Result r;
    r.time = c.timed([&] { hegst(1, Ah, Bh, c.opts); });
    r.flops = cfac<T>() * double(c.n) * c.n * c.n;
    if (c.P.check) {
        BaseTrapezoidMatrix<T> As(Uplo::Lower, A, MatrixKind::Trapezoid);
        auto F = full_of(c, As, true);
        TriangularMatrix<T> L(Uplo::Lower, Diag::NonUnit, Bg);
        trmm(Side::Left, T(1), L, F, c.opts);
        trmm(Side::Right, T(1), conj_transpose(L), F, c.opts);
        add(T(-1), A0, T(1), F, c.opts);
        r.error = c.nrm(F) / (double(c.n) * c.nrm(A0));
    }
    return r;
}

template <typename T>
Result r_getrs_v(Case<T>& c, int variant) {   // 0 getrs_nopiv, 1 getrs after tournament pivoting
    auto A = c.mat(c.n, c.n, variant == 0 ? "rands+n" : "rands", -1, true), B = c.mat(c.n, c.P.nrhs);
    auto A0 = c.copy_of(A), B0 = c.copy_of(B);
    Result r;
    Pivots piv;
    int64_t info = 0;
    if (variant == 0) info = getrf_nopiv(A, c.opts);
    else {
        Options o = c.opts;
        o[Option::MethodLU] = int64_t(MethodLU::CALU);
        info = getrf(A, piv, o);
    }
    if (info) { r.error = INFINITY; return r; }
    r.time = c.timed([&] {
        if (variant == 0) getrs_nopiv(A, B, c.opts);
        else getrs(A, piv, B, c.opts);
    });
    r.flops = cfac<T>() * 2.0 * c.n * c.n * c.P.nrhs;
    if (c.P.check) r.error = c.solve_resid(A0, B, B0);
    return r;
}

template <typename T>
Result r_scale_row_col(Case<T>& c) {
    using R = R_<T>;
    auto A = c.mat(c.m, c.n, "rands", -1, true);
    auto A0 = c.copy_of(A);
    std::vector<R> rs(c.m), cs(c.n), ri(c.m), ci(c.n);
    for (int64_t i = 0; i < c.m; ++i) { rs[i] = R(1) + R(i % 5) / R(4); ri[i] = R(1) / rs[i]; }
    for (int64_t j = 0; j < c.n; ++j) { cs[j] = R(2) - R(j % 3) / R(4); ci[j] = R(1) / cs[j]; }
    Result r;
    r.time = c.timed([&] { scale_row_col(Equed::Both, rs, cs, A, c.opts); });
    r.flops = 2.0 * double(c.m) * c.n;
    if (c.P.check) {
        scale_row_col(Equed::Both, ri, ci, A, c.opts);
        add(T(-1), A0, T(1), A, c.opts);
        r.error = c.nrm(A) / c.nrm(A0);
    }
    return r;
}

template <typename T>
Result r_norm_kind(Case<T>& c, int kind) {   // 0 gbnorm, 1 hbnorm, 2 synorm, 3 trnorm
    auto Ag = c.mat(c.n, c.n, "rands", -1, true);
    const int64_t kd = std::max<int64_t>(1, c.nb / 2);
    Result r;
    r.flops = double(c.n) * c.n;
    const Norm nt = Norm::One;
    R_<T> v = 0;
    double ref = 0;
    if (kind == 0) {
        BandMatrix<T> B(kd, kd / 2 + 1, Ag);
        r.time = c.timed([&] { v = norm(nt, B, c.opts); });
        if (c.P.check) ref = c.nrm(dense_band(c, B));
    } else if (kind == 1) {
        HermitianBandMatrix<T> H(Uplo::Lower, kd, Ag);
        r.time = c.timed([&] { v = norm(nt, H, c.opts); });
        if (c.P.check) {
            // lanhb reads only the real part of the diagonal
            auto F = dense_hband(c, H), Ft = c.zeros(c.n, c.n);
            copy<T, T>(conj_transpose(F), Ft, c.opts);
            add(T(0.5), Ft, T(0.5), F, c.opts);
            ref = c.nrm(F);
        }
    } else if (kind == 2) {
        SymmetricMatrix<T> S(c.P.uplo, Ag);
        r.time = c.timed([&] { v = norm(nt, S, c.opts); });
        if (c.P.check) {
            BaseTrapezoidMatrix<T> Ss(c.P.uplo, Ag, MatrixKind::Trapezoid);
            ref = c.nrm(full_of(c, Ss, false));
        }
    } else {
        TriangularMatrix<T> Tm(c.P.uplo, c.P.diag, Ag);
        r.time = c.timed([&] { v = norm(nt, Tm, c.opts); });
        if (c.P.check) {
            auto D = c.zeros(c.n, c.n);
            BaseTrapezoidMatrix<T> Ls(c.P.uplo, Ag, MatrixKind::Trapezoid), Ds(c.P.uplo, D, MatrixKind::Trapezoid);
            copy<T, T>(Ls, Ds, c.opts);
            if (c.P.diag == Diag::Unit) {
                // unit diagonal: D - diag(D) + I
                auto Dd = dense_diag(c, D);
                add(T(-1), Dd, T(1), D, c.opts);
                auto I = c.zeros(c.n, c.n);
                set(T(0), T(1), I, c.opts);
                add(T(1), I, T(1), D, c.opts);
            }
            ref = c.nrm(D);
        }
    }
    if (c.P.check) r.error = std::abs(double(v) - ref) / std::max(ref, 1e-300);
    return r;
}

/// trapezoid aux variants on the --uplo triangle: 0 set, 1 copy, 2 scale, 3 add;
/// kind: the view type name (tz / tr / sy / he) only selects the wrapper.
template <typename T>
Result r_tzaux(Case<T>& c, int op) {
    auto A = c.mat(c.m, c.n, "rands", -1, true), B = c.mat(c.m, c.n);
    std::vector<T> a0, b0;
    gather(A, a0, c.opts);
    gather(B, b0, c.opts);
    const Uplo u = c.P.uplo;
    BaseTrapezoidMatrix<T> At(u, A, MatrixKind::Trapezoid), Bt(u, B, MatrixKind::Trapezoid);
    Result r;
    r.flops = double(c.m) * c.n / 2;
    const T off(0.25), dg(3), al(2), be(-1);
    r.time = c.timed([&] {
        if (op == 0) set(off, dg, Bt, c.opts);
        else if (op == 1) copy<T, T>(At, Bt, c.opts);
        else if (op == 2) scale(R_<T>(3), R_<T>(2), Bt, c.opts);
        else add(al, At, be, Bt, c.opts);
    });
    if (c.P.check) {
        std::vector<T> b1;
        gather(B, b1, c.opts);
        double err = 0, mx = 1e-300;
        for (int64_t j = 0; j < c.n; ++j)
            for (int64_t i = 0; i < c.m; ++i) {
                const size_t x = size_t(i) + size_t(j) * c.m;
                const bool in = u == Uplo::Lower ? i >= j : i <= j;
                T want = b0[x];
                if (in) {
                    if (op == 0) want = i == j ? dg : off;
                    else if (op == 1) want = a0[x];
                    else if (op == 2) want = b0[x] * T(1.5);
                    else want = al * a0[x] + be * b0[x];
                }
                err = std::max(err, double(std::abs(b1[x] - want)));
                mx = std::max(mx, double(std::abs(want)));
            }
        r.error = err / mx;
    }
    return r;
}

template <typename T>
Result r_sy(Case<T>& c, int variant) {   // 0 sysv, 1 sytrf (+ sytrs for the check), 2 sytrs
    if constexpr (is_complex_v<T>) {
        Result r; r.skipped = true; r.note = "real types (use hesv/hetrf)"; return r;
    } else {
        auto S0 = herm_of(c, c.n);
        auto Sg = c.copy_of(S0), B = c.mat(c.n, c.P.nrhs);
        auto B0 = c.copy_of(B);
        SymmetricMatrix<T> S(Uplo::Lower, Sg);
        std::vector<int64_t> ipiv;
        Result r;
        int64_t info = 0;
        r.flops = double(c.n) * c.n * c.n / 3;
        if (variant == 0) r.time = c.timed([&] { info = sysv(S, ipiv, B, c.opts); });
        else if (variant == 1) {
            r.time = c.timed([&] { info = sytrf(S, ipiv, c.opts); });
            if (!info) sytrs(S, ipiv, B, c.opts);
        } else {
            info = sytrf(S, ipiv, c.opts);
            if (!info) r.time = c.timed([&] { sytrs(S, ipiv, B, c.opts); });
            r.flops = 2.0 * double(c.n) * c.n * c.P.nrhs;
        }
        if (info) { r.error = INFINITY; return r; }
        if (c.P.check) r.error = c.solve_resid(S0, B, B0);
        return r;
    }
}


template <typename T>
Result r_hetrs(Case<T>& c) {   // Bunch-Kaufman solve with an untimed hetrf (reference test_hesv.cc, hetrs)
    auto Ag = c.mat(c.n, c.n, "rands", -1, true), B = c.mat(c.n, c.P.nrhs);
    auto H0 = c.zeros(c.n, c.n);
    copy<T, T>(conj_transpose(Ag), H0, c.opts);
    add(T(1), Ag, T(1), H0, c.opts);
    auto Hg = c.copy_of(H0), B0 = c.copy_of(B);
    HermitianMatrix<T> H(Uplo::Lower, Hg);
    std::vector<int64_t> ipiv;
    Result r;
    if (hetrf(H, ipiv, c.opts)) { r.error = INFINITY; return r; }
    r.time = c.timed([&] { hetrs(H, ipiv, B, c.opts); });
    r.flops = cfac<T>() * 2.0 * double(c.n) * c.n * c.P.nrhs;
    if (c.P.check) r.error = c.solve_resid(H0, B, B0);
    return r;
}

/// D&C stages on their own (reference test_stedc_{z_vector,sort,deflate,
/// secular}.cc).  Each checks its defining property on the host:
///   0 z_vector: z = [Q(n1-1, 0:n1); sgn Q(n1, n1:n)] / sqrt 2
///   1 sort:     D ascending, (D, z, Q columns) permuted consistently
///   2 deflate:  Q (diag(D) + rho z z^T) Q^T invariant, deflated z ~ 0
///   3 secular:  (diag(D) + rho z z^T) U = U diag(Lambda), U orthogonal
template <typename T>
Result r_stedc_stage(Case<T>& c, int stage) {
    using R = R_<T>;
    Result r;
    if constexpr (is_complex_v<T>) {
        r.skipped = true; r.note = "real types (stedc works on R)"; return r;
    } else {
        const int64_t n = c.n, n1 = n / 2;
        const R eps = std::numeric_limits<R>::epsilon();
        auto hv = [](int64_t i, uint64_t salt) {   // deterministic values in [-1, 1)
            uint64_t x = (uint64_t(i) + 1) * 0x9E3779B97F4A7C15ull ^ (salt * 0xBF58476D1CE4E5B9ull);
            x ^= x >> 31; x *= 0x94D049BB133111EBull; x ^= x >> 29;
            return R(double(x >> 11) / double(1ull << 53) * 2.0 - 1.0);
        };
        auto Q = c.zeros(n, n);
        std::vector<T> q0, q1;
        if (stage == 0) {
            std::function<T(int64_t, int64_t)> qv = [&](int64_t i, int64_t j) -> T { return T(hv(i * n + j, 1)); };
            set(qv, Q, c.opts);
            std::vector<R> z;
            r.time = c.timed([&] { stedc_z_vector(Q, n1, R(-1), z, c.opts); });
            double err = 0;
            for (int64_t j = 0; j < n; ++j) {
                R want = (j < n1 ? hv((n1 - 1) * n + j, 1) : -hv(n1 * n + j, 1)) / std::sqrt(R(2));
                err = std::max(err, double(std::abs(z[j] - want)));
            }
            r.error = err;
            r.flops = double(n);
            return r;
        }
        if (stage == 1) {
            std::function<T(int64_t, int64_t)> qv = [&](int64_t i, int64_t j) -> T { return T(hv(i * n + j, 2)); };
            set(qv, Q, c.opts);
            std::vector<R> D(n), z(n);
            for (int64_t j = 0; j < n; ++j) { D[j] = hv(j, 3); z[j] = hv(j, 4); }
            auto D0 = D; auto z0 = z;
            auto Qo = c.zeros(n, n);
            std::vector<int64_t> perm;
            gather(Q, q0, c.opts);
            r.time = c.timed([&] { stedc_sort(D, z, Q, Qo, perm, c.opts); });
            gather(Qo, q1, c.opts);
            double err = 0;
            for (int64_t j = 0; j < n; ++j) {
                if (j > 0 && D[j] < D[j - 1]) err = INFINITY;
                err = std::max(err, double(std::abs(D[j] - D0[perm[j]]) + std::abs(z[j] - z0[perm[j]])));
                for (int64_t i = 0; i < n; ++i)
                    err = std::max(err, double(std::abs(q1[i + j * n] - q0[i + perm[j] * n])));
            }
            r.error = err;
            r.flops = double(n) * n;
            return r;
        }
        // rank-one modified diagonal: sorted D with clusters (pairs within
        // ~eps) and a few tiny z entries, so the deflation paths all run
        std::vector<R> D(n), z(n);
        for (int64_t j = 0; j < n; ++j) D[j] = R(j / 2) + ((j % 2) ? R(4) * eps : R(0)) + R(0.25) * R(j % 3 == 0);
        std::sort(D.begin(), D.end());
        R zn = 0;
        for (int64_t j = 0; j < n; ++j) { z[j] = (j % 11 == 5) ? R(1e-20) : R(0.5) + R(0.5) * std::abs(hv(j, 5)); zn += z[j] * z[j]; }
        for (auto& x : z) x /= std::sqrt(zn);
        const R rho = R(1.5);
        auto M = [&](std::vector<R> const& d, std::vector<R> const& zz) {
            std::vector<R> m(size_t(n) * n, R(0));
            for (int64_t j = 0; j < n; ++j) {
                for (int64_t i = 0; i < n; ++i) m[i + j * n] = rho * zz[i] * zz[j];
                m[j + j * n] += d[j];
            }
            return m;
        };
        const auto M0 = M(D, z);
        double m0 = 0;
        for (auto v : M0) m0 = std::max(m0, double(std::abs(v)));
        if (stage == 2) {
            set(T(0), T(1), Q, c.opts);
            std::vector<char> defl;
            int64_t k = 0;
            r.time = c.timed([&] { k = stedc_deflate(rho, D, z, Q, defl, c.opts); });
            gather(Q, q1, c.opts);
            const auto M1 = M(D, z);
            // Q M1 Q^T - M0
            double err = 0;
            std::vector<R> QM(size_t(n) * n, R(0));
            for (int64_t j = 0; j < n; ++j)
                for (int64_t l = 0; l < n; ++l) {
                    R b = M1[l + j * n];
                    if (b == R(0)) continue;
                    for (int64_t i = 0; i < n; ++i) QM[i + j * n] += R(q1[i + l * n]) * b;
                }
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = 0; i < n; ++i) {
                    R v = 0;
                    for (int64_t l = 0; l < n; ++l) v += QM[i + l * n] * R(q1[j + l * n]);
                    err = std::max(err, double(std::abs(v - M0[i + j * n])));
                }
            int64_t nd = 0;
            for (int64_t j = 0; j < n; ++j) if (defl[j]) { ++nd; err = std::max(err, double(rho * std::abs(z[j])) / 64); }
            if (nd + k != n || nd == 0) err = INFINITY;   // the test matrix must deflate something
            r.error = err / (m0 * double(n));
            r.flops = double(n) * n;
            return r;
        }
        // secular: strictly separated D, no deflation
        for (int64_t j = 0; j < n; ++j) D[j] = R(j) + R(0.1) * hv(j, 6);
        for (int64_t j = 0; j < n; ++j) z[j] = R(0.2) + std::abs(hv(j, 7));
        const auto Ms = M(D, z);
        double ms = 0;
        for (auto v : Ms) ms = std::max(ms, double(std::abs(v)));
        std::vector<R> lam;
        auto U = c.zeros(n, n);
        r.time = c.timed([&] { stedc_secular(rho, D, z, lam, U, c.opts); });
        gather(U, q1, c.opts);
        double err = 0, orth = 0;
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < n; ++i) {
                R v = 0, o = 0;
                for (int64_t l = 0; l < n; ++l) {
                    v += Ms[i + l * n] * R(q1[l + j * n]);
                    o += R(q1[l + i * n]) * R(q1[l + j * n]);
                }
                err = std::max(err, double(std::abs(v - lam[j] * R(q1[i + j * n]))));
                orth = std::max(orth, double(std::abs(o - (i == j ? R(1) : R(0)))));
            }
        r.error = std::max(err / ms, orth) / double(n);
        r.flops = 4.0 * double(n) * n;
        return r;
    }
}

template <typename T>
using Fn = std::function<Result(Case<T>&)>;

template <typename T>
std::map<std::string, Fn<T>> routines() {
    return {
        {"gemm", r_gemm<T>}, {"herk", r_herk<T>}, {"hemm", r_hemm<T>}, {"trsm", r_trsm<T>}, {"trmm", r_trmm<T>},
        {"getrf", [](Case<T>& c) { return r_getrf_m<T>(c, MethodLU::PartialPiv); }},
        {"getrf_tntpiv", [](Case<T>& c) { return r_getrf_m<T>(c, MethodLU::CALU); }},
        {"getrf_nopiv", r_getrf_nopiv<T>}, {"gesv", r_gesv<T>},
        {"gesv_mixed", [](Case<T>& c) { return r_gesv_mixed_v<T>(c, 0); }},
        {"gesv_mixed_gmres", [](Case<T>& c) { return r_gesv_mixed_v<T>(c, 1); }},
        {"posv_mixed", [](Case<T>& c) { return r_gesv_mixed_v<T>(c, 2); }},
        {"potrf", [](Case<T>& c) { return r_posv<T>(c, true); }},
        {"posv", [](Case<T>& c) { return r_posv<T>(c, false); }},
        {"getri", r_getri<T>}, {"trtri", r_trtri<T>},
        {"geqrf", r_geqrf<T>}, {"gelqf", r_gelqf<T>}, {"gels", r_gels<T>},
        {"heev", r_heev<T>}, {"svd", r_svd<T>}, {"hesv", r_hesv<T>}, {"gbsv", r_gbsv<T>}, {"genorm", r_genorm<T>},
        {"syrk", [](Case<T>& c) { return r_rankk<T>(c, 0); }},
        {"her2k", [](Case<T>& c) { return r_rankk<T>(c, 1); }},
        {"syr2k", [](Case<T>& c) { return r_rankk<T>(c, 2); }},
        {"symm", r_symm<T>},
        {"gemmA", [](Case<T>& c) { return r_gemm_m<T>(c, MethodGemm::GemmA); }},
        {"gemmC", [](Case<T>& c) { return r_gemm_m<T>(c, MethodGemm::GemmC); }},
        {"getrs", r_getrs<T>},
        {"potrs", [](Case<T>& c) { return r_potrs<T>(c, 0); }},
        {"potri", [](Case<T>& c) { return r_potrs<T>(c, 1); }},
        {"gesv_nopiv", [](Case<T>& c) { return r_gesv_v<T>(c, 0); }},
        {"gesv_tntpiv", [](Case<T>& c) { return r_gesv_v<T>(c, 1); }},
        {"gesv_rbt", [](Case<T>& c) { return r_gesv_v<T>(c, 2); }},
        {"gecondest", [](Case<T>& c) { return r_condest<T>(c, 0); }},
        {"pocondest", [](Case<T>& c) { return r_condest<T>(c, 1); }},
        {"trcondest", [](Case<T>& c) { return r_condest<T>(c, 2); }},
        {"unmqr", [](Case<T>& c) { return r_unmqr<T>(c, false); }},
        {"unmlq", [](Case<T>& c) { return r_unmqr<T>(c, true); }},
        {"cholqr", r_cholqr<T>},
        {"gbtrf", [](Case<T>& c) { return r_band<T>(c, 0); }},
        {"pbsv", [](Case<T>& c) { return r_band<T>(c, 1); }},
        {"pbtrf", [](Case<T>& c) { return r_band<T>(c, 2); }},
        {"gbmm", [](Case<T>& c) { return r_band<T>(c, 3); }},
        {"hbmm", [](Case<T>& c) { return r_band<T>(c, 4); }},
        {"tbsm", [](Case<T>& c) { return r_band<T>(c, 5); }},
        {"tbsm_pivots", [](Case<T>& c) { return r_band<T>(c, 8); }},
        {"hetrf", r_hetrf<T>},
        {"hesv_aasen", r_hesv_aasen<T>},
        {"heev_vals", [](Case<T>& c) { return r_vals<T>(c, 0); }},
        {"svd_vals", [](Case<T>& c) { return r_vals<T>(c, 1); }},
        {"hegv", [](Case<T>& c) { return r_vals<T>(c, 2); }},
        {"sterf", [](Case<T>& c) { return r_tridiag<T>(c, 0); }},
        {"steqr2", [](Case<T>& c) { return r_tridiag<T>(c, 1); }},
        {"add", [](Case<T>& c) { return r_aux<T>(c, 0); }},
        {"copy", [](Case<T>& c) { return r_aux<T>(c, 1); }},
        {"scale", [](Case<T>& c) { return r_aux<T>(c, 2); }},
        {"set", [](Case<T>& c) { return r_aux<T>(c, 3); }},
        {"trtrm", [](Case<T>& c) { return r_aux<T>(c, 4); }},
        {"colnorms", [](Case<T>& c) { return r_aux<T>(c, 5); }},
        {"henorm", [](Case<T>& c) { return r_aux<T>(c, 6); }},
        {"redistribute", [](Case<T>& c) { return r_aux<T>(c, 7); }},
        {"he2hb", [](Case<T>& c) { return r_he2hb<T>(c, 0); }},
        {"unmtr_he2hb", [](Case<T>& c) { return r_he2hb<T>(c, 1); }},
        {"hb2st", [](Case<T>& c) { return r_hb2st<T>(c, 0); }},
        {"unmtr_hb2st", [](Case<T>& c) { return r_hb2st<T>(c, 1); }},
        {"ge2tb", r_ge2tb<T>},
        {"tb2bd", [](Case<T>& c) { return r_tb2bd<T>(c, 0); }},
        {"unmbr_tb2bd", [](Case<T>& c) { return r_tb2bd<T>(c, 1); }},
        {"bdsqr", r_bdsqr<T>},
        {"stedc", r_stedc<T>},
        {"hegst", r_hegst<T>},
        {"getrs_nopiv", [](Case<T>& c) { return r_getrs_v<T>(c, 0); }},
        {"getrs_tntpiv", [](Case<T>& c) { return r_getrs_v<T>(c, 1); }},
        {"posv_mixed_gmres", [](Case<T>& c) { return r_gesv_mixed_v<T>(c, 3); }},
        {"gbtrs", [](Case<T>& c) { return r_band<T>(c, 6); }},
        {"pbtrs", [](Case<T>& c) { return r_band<T>(c, 7); }},
        {"scale_row_col", r_scale_row_col<T>},
        {"gbnorm", [](Case<T>& c) { return r_norm_kind<T>(c, 0); }},
        {"hbnorm", [](Case<T>& c) { return r_norm_kind<T>(c, 1); }},
        {"synorm", [](Case<T>& c) { return r_norm_kind<T>(c, 2); }},
        {"trnorm", [](Case<T>& c) { return r_norm_kind<T>(c, 3); }},
        {"tzset", [](Case<T>& c) { return r_tzaux<T>(c, 0); }},
        {"tzcopy", [](Case<T>& c) { return r_tzaux<T>(c, 1); }},
        {"tzscale", [](Case<T>& c) { return r_tzaux<T>(c, 2); }},
        {"tzadd", [](Case<T>& c) { return r_tzaux<T>(c, 3); }},
        {"trset", [](Case<T>& c) { return r_tzaux<T>(c, 0); }},
        {"trcopy", [](Case<T>& c) { return r_tzaux<T>(c, 1); }},
        {"trscale", [](Case<T>& c) { return r_tzaux<T>(c, 2); }},
        {"tradd", [](Case<T>& c) { return r_tzaux<T>(c, 3); }},
        {"syset", [](Case<T>& c) { return r_tzaux<T>(c, 0); }},
        {"sycopy", [](Case<T>& c) { return r_tzaux<T>(c, 1); }},
        {"syscale", [](Case<T>& c) { return r_tzaux<T>(c, 2); }},
        {"syadd", [](Case<T>& c) { return r_tzaux<T>(c, 3); }},
        {"heset", [](Case<T>& c) { return r_tzaux<T>(c, 0); }},
        {"hecopy", [](Case<T>& c) { return r_tzaux<T>(c, 1); }},
        {"hescale", [](Case<T>& c) { return r_tzaux<T>(c, 2); }},
        {"headd", [](Case<T>& c) { return r_tzaux<T>(c, 3); }},
        {"sysv", [](Case<T>& c) { return r_sy<T>(c, 0); }},
        {"sytrf", [](Case<T>& c) { return r_sy<T>(c, 1); }},
        {"sytrs", [](Case<T>& c) { return r_sy<T>(c, 2); }},
        {"hetrs", r_hetrs<T>},
        {"stedc_z_vector", [](Case<T>& c) { return r_stedc_stage<T>(c, 0); }},
        {"stedc_sort", [](Case<T>& c) { return r_stedc_stage<T>(c, 1); }},
        {"stedc_deflate", [](Case<T>& c) { return r_stedc_stage<T>(c, 2); }},
        {"stedc_secular", [](Case<T>& c) { return r_stedc_stage<T>(c, 3); }},
    };
}

template <typename T>
double eps_of() { return double(std::numeric_limits<R_<T>>::epsilon()); }

template <typename T>
int run_type(Params const& P, char tc, std::string const& name) {
    auto table = routines<T>();
    auto it = table.find(name);
    if (it == table.end()) {
        if (rank() == 0) std::fprintf(stderr, "unknown routine %s\n", name.c_str());
        return 1;
    }
    int fails = 0;
    auto g = default_grid();
    for (auto const& d : P.dims)
        for (int64_t nb : P.nbs)
            for (int rep = 0; rep < P.repeat; ++rep) {
                Case<T> c(P, d, nb);
                Result r;
                std::string status;
                try {
                    r = it->second(c);
                    if (r.skipped) status = "skip (" + r.note + ")";
                    else {
                        bool ok = !P.check || r.error <= P.tol * eps_of<T>();
                        status = ok ? "pass" : "FAILED";
                        fails += !ok;
                    }
                } catch (std::exception const& e) {
                    status = std::string("FAILED: ") + e.what();
                    ++fails;
                }
                if (rank() == 0) {
                    char es[32];
                    if (P.check && !r.skipped && !std::isnan(r.error)) std::snprintf(es, sizeof(es), "%10.2e", r.error);
                    else std::snprintf(es, sizeof(es), "%10s", "NA");
                    double gf = (r.time > 0 && r.flops > 0) ? r.flops / r.time / 1e9 : NAN;
                    std::printf("%-16s %-4c %7lld %7lld %7lld %5lld %2d %2d %s %10.4f %11.2f  %s%s%s\n", name.c_str(), tc,
                                (long long)c.m, (long long)c.n, (long long)c.k, (long long)nb, g->p(), g->q(), es,
                                r.time, gf, status.c_str(), (r.note.empty() || r.skipped) ? "" : "  ",
                                r.skipped ? "" : r.note.c_str());
                    std::fflush(stdout);
                }
                if (P.timer_level >= 2) {
                    // per-driver wall time of this case from the host trace (reference --timer-level 2)
                    std::map<std::string, double> tot;
                    for (auto const& e : trace::Trace::events())
                        if (e.lane < 100) tot[e.name] += e.stop - e.start;
                    if (rank() == 0)
                        for (auto const& kv : tot) std::printf("#   %-24s %10.4f s\n", kv.first.c_str(), kv.second);
                    trace::Trace::clear();
                }
            }
    return fails;
}

void usage() {
    std::printf(
        "usage: slate_tester ROUTINE[,ROUTINE...]|all [--type d,s,z,c] [--dim N|A:B:STEP|MxNxK,...]\n"
        "       [--nb NB,...] [--grid PxQ] [--target d|h] [--lookahead LA] [--nrhs K]\n"
        "       [--check y|n] [--tol T] [--repeat R] [--trace y|n]\n"
        "       [--matrix KIND] [--method-lu ppiv|calu|nopiv] [--method-trsm auto|A|B]\n"
        "       [--method-gemm auto|A|C] [--method-hemm auto|A|C] [--method-cholqr auto|herkC|gemmA|gemmC]\n"
        "       [--origin h|d]\n"
        "       [--timer-level 1|2] [--itermax N] [--fallback y|n] [--pivot-threshold X]\n"
        "       [--uplo l|u] [--trans n|t|c] [--side l|r] [--diag n|u] [--cond C] [--ib IB]\n"
        "       [--nonuniform-nb y|n] [--go c|r] [--do r|c]\n"
        "routines:");
    for (auto const& kv : routines<double>()) std::printf(" %s", kv.first.c_str());
    std::printf("\n");
}

}  // namespace

int main(int argc, char** argv) {
    Params P;
    std::string rlist;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto val = [&]() -> std::string {
            if (i + 1 >= argc) { usage(); std::exit(2); }
            return argv[++i];
        };
        if (a == "-h" || a == "--help") { usage(); return 0; }
        else if (a == "--type") P.types = val();
        else if (a == "--dim") P.dims = parse_dims(val());
        else if (a == "--nb") P.nbs = parse_list(val());
        else if (a == "--grid") {
            std::string g = val();
            P.p = std::stoi(g.substr(0, g.find('x')));
            P.q = std::stoi(g.substr(g.find('x') + 1));
        }
        else if (a == "--target") { std::string t = val(); P.target = (t[0] == 'd' || t[0] == 'D') ? Target::Devices : Target::HostTask; }
        else if (a == "--lookahead" || a == "--la") P.lookahead = std::stoll(val());
        else if (a == "--nrhs") P.nrhs = std::stoll(val());
        else if (a == "--check") P.check = val()[0] == 'y';
        else if (a == "--tol") P.tol = std::stod(val());
        else if (a == "--repeat") P.repeat = std::stoi(val());
        else if (a == "--trace") P.trace = val()[0] == 'y';
        else if (a == "--matrix") P.matrix = val();
        else if (a == "--method-lu") P.method_lu = MethodLU::str2method(val());
        else if (a == "--method-trsm") P.method_trsm = MethodTrsm::str2method(val());
        else if (a == "--method-gemm") P.method_gemm = MethodGemm::str2method(val());
        else if (a == "--method-hemm") P.method_hemm = MethodHemm::str2method(val());
        else if (a == "--method-cholqr") P.method_cholqr = MethodCholQR::str2method(val());
        else if (a == "--origin") P.origin = char(std::tolower(val()[0]));
        else if (a == "--timer-level") P.timer_level = std::stoi(val());
        else if (a == "--itermax") P.itermax = std::stoll(val());
        else if (a == "--fallback") P.fallback = val()[0] == 'y' ? 1 : 0;
        else if (a == "--pivot-threshold") P.pivot_threshold = std::stod(val());
        else if (a == "--uplo") { char v = char(std::tolower(val()[0])); P.uplo = v == 'u' ? Uplo::Upper : Uplo::Lower; }
        else if (a == "--trans") {
            char v = char(std::tolower(val()[0]));
            P.trans = v == 't' ? Op::Trans : (v == 'c' ? Op::ConjTrans : Op::NoTrans);
        }
        else if (a == "--side") P.side = char(std::tolower(val()[0])) == 'r' ? Side::Right : Side::Left;
        else if (a == "--diag") P.diag = char(std::tolower(val()[0])) == 'u' ? Diag::Unit : Diag::NonUnit;
        else if (a == "--cond") P.cond = std::stod(val());
        else if (a == "--ib") P.ib = std::stoll(val());
        else if (a == "--nonuniform-nb") P.nonuniform = val()[0] == 'y';
        else if (a == "--go") P.order = char(std::tolower(val()[0])) == 'r' ? GridOrder::Row : GridOrder::Col;
        else if (a == "--do") P.dev_order = char(std::tolower(val()[0]));
        else if (!a.empty() && a[0] != '-') rlist = rlist.empty() ? a : rlist + "," + a;
        else { usage(); return 2; }
    }
    if (rlist.empty()) { usage(); return 2; }
    init_grid(P.p, P.q, P.order);
    if (rlist == "all") {
        rlist.clear();
        for (auto const& kv : routines<double>()) rlist += (rlist.empty() ? "" : ",") + kv.first;
    }
    if (rank() == 0) {
        std::printf("# slate %s tester: %d process(es), grid %dx%d, target %s\n", version(), default_grid()->size(),
                    default_grid()->p(), default_grid()->q(), P.target == Target::Devices ? "devices" : "host");
        std::printf("%-16s %-4s %7s %7s %7s %5s %2s %2s %10s %10s %11s  %s\n", "routine", "type", "m", "n", "k", "nb",
                    "p", "q", "error", "time(s)", "gflop/s", "status");
    }
    if (P.trace || P.timer_level >= 2) trace::Trace::on();
    int fails = 0;
    std::stringstream rs(rlist);
    std::string name;
    while (std::getline(rs, name, ','))
        for (char tc : P.types) {
            switch (tc) {
                case 's': fails += run_type<float>(P, tc, name); break;
                case 'd': fails += run_type<double>(P, tc, name); break;
                case 'c': fails += run_type<std::complex<float>>(P, tc, name); break;
                case 'z': fails += run_type<std::complex<double>>(P, tc, name); break;
                default: break;
            }
        }
    if (P.trace) trace::Trace::finish(&default_grid()->world());
    int total = int(default_grid()->world().allreduce_scalar<int32_t>(fails, ReduceOp::Sum));
    if (rank() == 0) std::printf(total ? "# %d failed\n" : "# all tests passed\n", total);
    finalize();
    return total ? 1 : 0;
}
