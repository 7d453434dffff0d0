// Test-matrix generation driver (reference matgen/generate_matrix_utils.cc:64-420
// decode, generate_matrix_ge.cc:37-300 kinds, generate_sigma.hh, generate_type_svd.hh,
// generate_type_heev.hh, generate_matrix_he_and_tz.cc).
//
// Element kinds are evaluated in one pass over the local block-cyclic array
// (device kernel in kernels/matgen.hip, or a host OpenMP loop) from the
// formulas in kernels/matgen_entry.hh, so every grid and target yields the
// same matrix.  Spectral kinds (svd / poev / heev / geev) build
// A = Q1 * D * Q2^H with Householder Q's from this library's own distributed
// geqrf / unmqr on random normal matrices, as the reference does.
#include "internal.hh"
#include "slate_amd/matgen.hh"
#include "slate_amd/slate.hh"
#include "../kernels/kernels.hh"

#include <cstdio>
#include <cstdlib>
#include <stdexcept>

namespace slate {

namespace gen = slate_amd::gen;

namespace {

enum class Dist {
    None, Rand, Rands, Randn, Logrand, Arith, Geo, Cluster0, Cluster1, Rarith, Rgeo, Rcluster0, Rcluster1, Specified,
};
enum class Spectral { None, Diag, Svd, Poev, Heev, Geev, Geevx };

struct Decoded {
    int code = gen::Rands;
    Spectral spec = Spectral::None;
    Dist dist = Dist::None;
    double cond = 0, condD = 1, sigma_max = 1;
    bool dominant = false;
    int64_t zero_col = -1;
};

std::vector<std::string> split(std::string const& s, std::string const& delims) {
    std::vector<std::string> out;
    size_t start = 0;
    while (true) {
        size_t e = s.find_first_of(delims, start);
        out.push_back(s.substr(start, e == std::string::npos ? std::string::npos : e - start));
        if (e == std::string::npos) break;
        start = e + 1;
    }
    return out;
}

[[noreturn]] void bad(std::string const& kind, std::string const& what) {
    throw Exception("generate_matrix: in '" + kind + "': " + what);
}

template <typename R>
Decoded decode(MatgenParams& params, int64_t m, int64_t n) {
    const double ufl = double(std::numeric_limits<R>::min());
    const double ofl = 1 / ufl;
    const double eps = double(std::numeric_limits<R>::epsilon());
    Decoded d;
    std::string const& kind = params.kind;
    d.cond = std::isnan(params.cond_request) ? 1 / std::sqrt(eps) : params.cond_request;
    bool condD_default = std::isnan(params.condD);
    d.condD = condD_default ? 1 : params.condD;

    auto tok = split(kind, "-_");
    std::string base = tok.empty() ? "" : tok[0];
    static const std::pair<const char*, int> elem[] = {
        {"zeros", gen::Zeros}, {"ones", gen::Ones}, {"identity", gen::Identity}, {"ij", gen::Ij},
        {"jordan", gen::Jordan}, {"jordanT", gen::JordanT}, {"chebspec", gen::Chebspec}, {"circul", gen::Circul},
        {"fiedler", gen::Fiedler}, {"gfpp", gen::Gfpp}, {"kms", gen::Kms}, {"orthog", gen::Orthog},
        {"riemann", gen::Riemann}, {"ris", gen::Ris}, {"zielkeNS", gen::ZielkeNS}, {"rand", gen::Rand},
        {"rands", gen::Rands}, {"randn", gen::Randn}, {"randb", gen::Randb}, {"randr", gen::Randr},
    };
    bool found = false;
    for (auto& e : elem) if (base == e.first) { d.code = e.second; found = true; }
    if (!found) {
        if (base == "diag") d.spec = Spectral::Diag;
        else if (base == "svd") d.spec = Spectral::Svd;
        else if (base == "poev" || base == "spd") d.spec = Spectral::Poev;
        else if (base == "heev" || base == "syev") d.spec = Spectral::Heev;
        else if (base == "geev") d.spec = Spectral::Geev;
        else if (base == "geevx") d.spec = Spectral::Geevx;
        else bad(kind, "unknown matrix '" + base + "'");
        d.code = gen::Diag;
    }
    static const std::pair<const char*, Dist> dists[] = {
        {"randn", Dist::Randn}, {"rands", Dist::Rands}, {"rand", Dist::Rand}, {"logrand", Dist::Logrand},
        {"arith", Dist::Arith}, {"geo", Dist::Geo}, {"cluster0", Dist::Cluster0}, {"cluster1", Dist::Cluster1},
        {"rarith", Dist::Rarith}, {"rgeo", Dist::Rgeo}, {"rcluster0", Dist::Rcluster0},
        {"rcluster1", Dist::Rcluster1}, {"specified", Dist::Specified},
    };
    for (size_t t = 1; t < tok.size(); ++t) {
        std::string const& s = tok[t];
        bool hit = false;
        for (auto& e : dists) if (s == e.first) { d.dist = e.second; hit = true; }
        if (hit) continue;
        if (s == "small") d.sigma_max = std::sqrt(ufl);
        else if (s == "large") d.sigma_max = std::sqrt(ofl);
        else if (s == "ufl") d.sigma_max = ufl;
        else if (s == "ofl") d.sigma_max = ofl;
        else if (s == "dominant") d.dominant = true;
        else if (s.rfind("zerocol", 0) == 0) {
            std::string num = s.substr(7);
            char* end = nullptr;
            double v = std::strtod(num.c_str(), &end);
            if (num.empty() || *end) bad(kind, "can't parse number after 'zerocol'");
            if (num.find('.') != std::string::npos) {
                if (v < 0 || v > 1) bad(kind, "fraction outside [0.0, 1.0]");
                d.zero_col = int64_t(v * double(n - 1));
            } else {
                d.zero_col = int64_t(v);
            }
            if (d.zero_col < 0 || d.zero_col >= n) bad(kind, "zerocol index outside [0, n)");
        } else {
            bad(kind, "unknown suffix '" + s + "'");
        }
    }
    const bool randkind = d.spec == Spectral::None && d.code >= gen::Rand && d.code <= gen::Randr;
    const bool spectral = d.spec != Spectral::None && d.spec != Spectral::Diag;
    if (d.dist != Dist::None && d.spec == Spectral::None) bad(kind, "matrix '" + base + "' doesn't support distribution");
    if (d.dist == Dist::None) d.dist = Dist::Logrand;
    if (d.sigma_max != 1 && !(randkind || spectral)) bad(kind, "matrix '" + base + "' doesn't support scaling");
    if (d.dominant && !(randkind || spectral)) bad(kind, "matrix '" + base + "' doesn't support diagonally dominant");
    if (m != n && (d.spec == Spectral::Poev || d.spec == Spectral::Heev || d.spec == Spectral::Geev ||
                   d.spec == Spectral::Geevx))
        bad(kind, "matrix '" + base + "' requires m == n");
    if (d.spec == Spectral::Geevx) bad(kind, "geevx not implemented");

    if (d.code == gen::Zeros || d.code == gen::Ones || d.zero_col >= 0) params.cond_actual = INFINITY;
    else if (d.code == gen::Identity || d.code == gen::Orthog) params.cond_actual = 1;
    else if (d.spec != Spectral::None) params.cond_actual = d.cond;
    else params.cond_actual = NAN;
    if (!condD_default && !(d.spec == Spectral::Svd || d.spec == Spectral::Heev || d.spec == Spectral::Poev))
        std::fprintf(stderr, "Warning: matrix '%s' ignores condD %.2e.\n", kind.c_str(), params.condD);
    if (d.spec == Spectral::Poev && (d.dist == Dist::Rands || d.dist == Dist::Randn))
        std::fprintf(stderr, "Warning: matrix '%s' using rands or randn will not generate SPD matrix; "
                             "use rand instead.\n", kind.c_str());
    return d;
}

/// Singular values / eigenvalues (reference generate_sigma.hh).
void make_sigma(Decoded const& d, bool rand_sign, uint64_t seed, std::vector<double>& S) {
    const int64_t k = int64_t(S.size());
    const double c = d.cond;
    auto frac = [&](int64_t i) { return k > 1 ? double(i) / double(k - 1) : 0.0; };
    switch (d.dist) {
        case Dist::Arith: for (int64_t i = 0; i < k; ++i) S[i] = 1 - frac(i) * (1 - 1 / c); break;
        case Dist::Rarith: for (int64_t i = 0; i < k; ++i) S[i] = 1 - frac(k - 1 - i) * (1 - 1 / c); break;
        case Dist::Geo: for (int64_t i = 0; i < k; ++i) S[i] = std::pow(c, -frac(i)); break;
        case Dist::Rgeo: for (int64_t i = 0; i < k; ++i) S[i] = std::pow(c, -frac(k - 1 - i)); break;
        case Dist::Cluster0: for (int64_t i = 0; i < k; ++i) S[i] = i == 0 ? 1 : 1 / c; break;
        case Dist::Rcluster0: for (int64_t i = 0; i < k; ++i) S[i] = i == k - 1 ? 1 : 1 / c; break;
        case Dist::Cluster1: for (int64_t i = 0; i < k; ++i) S[i] = i == k - 1 ? 1 / c : 1; break;
        case Dist::Rcluster1: for (int64_t i = 0; i < k; ++i) S[i] = i == 0 ? 1 / c : 1; break;
        case Dist::Logrand: {
            const double range = std::log(1 / c);
            for (int64_t i = 0; i < k; ++i) S[i] = std::exp(gen::rand_sample(gen::Rand, i, 0, seed) * range);
            if (k >= 2) { S[0] = 1; S[1] = 1 / c; }  // exact cond
            break;
        }
        case Dist::Rand: case Dist::Rands: case Dist::Randn: {
            int code = d.dist == Dist::Rand ? gen::Rand : d.dist == Dist::Rands ? gen::Rands : gen::Randn;
            for (int64_t i = 0; i < k; ++i) S[i] = gen::rand_sample(code, i, 0, seed);
            break;
        }
        case Dist::Specified: return;  // caller's values, unscaled
        case Dist::None: break;
    }
    if (d.sigma_max != 1) for (auto& s : S) s *= d.sigma_max;
    if (rand_sign)
        for (int64_t i = 0; i < k; ++i)
            if (gen::rand_sample(gen::Rand, i, 1, seed) > 0.5) S[i] = -S[i];
}

/// Evaluate `spec` on every local element of view A at the target location.
template <typename T>
void fill(gen::Spec spec, BaseMatrix<T>& A, Target target, std::vector<double> const* sigma = nullptr) {
    slate_error_if_msg(A.op() != Op::NoTrans, "generate_matrix: NoTrans view required");
    auto& s = *A.storage();
    auto& g = *s.grid;
    Loc loc = internal::loc_of(target);
    if (s.banded) {
        // band-only storage: the stored band elements on the host (the same
        // grid-independent values as a dense matrix), then the device
        spec.m = A.m(); spec.n = A.n(); spec.max_mn = std::max(A.m(), A.n());
        if (sigma) spec.sigma = sigma->data();
        using R = real_type<T>;
        internal::for_each_stored(A, true, [&](int64_t gi, int64_t gj, T& v) {
            double re, im;
            gen::entry(spec, gi, gj, is_complex_v<T>, re, im);
            if constexpr (is_complex_v<T>) v = T(R(re), R(im));
            else v = T(re);
        });
        if (target == Target::Devices) s.get(Loc::Device, false);
        return;
    }
    if (s.general()) {
        // arbitrary distribution (non-uniform tiles, any owner map): my tiles
        // one by one on the host with the same grid-independent values, then
        // the device instance
        spec.m = A.m(); spec.n = A.n(); spec.max_mn = std::max(A.m(), A.n());
        if (sigma) spec.sigma = sigma->data();
        using R = real_type<T>;
        slate_error_if_msg(A.row0() != 0 || A.col0() != 0, "generate_matrix: arbitrary layouts need the whole matrix");
        s.get(Loc::Host, true);
        for (int64_t j = 0; j < A.nt(); ++j)
            for (int64_t i = 0; i < A.mt(); ++i) {
                if (!A.tileIsLocal(i, j)) continue;
                Tile<T> t = A.tile(i, j, Loc::Host);
                const int64_t gi0 = s.layout->rs[i], gj0 = s.layout->cs[j];
                for (int64_t jj = 0; jj < t.nb; ++jj)
                    for (int64_t ii = 0; ii < t.mb; ++ii) {
                        double re, im;
                        gen::entry(spec, gi0 + ii, gj0 + jj, is_complex_v<T>, re, im);
                        if constexpr (is_complex_v<T>) t.data[ii + jj * t.stride] = T(R(re), R(im));
                        else t.data[ii + jj * t.stride] = T(re);
                    }
            }
        if (target == Target::Devices) s.get(Loc::Device, false);
        return;
    }
    LocalBlock<T> lb = A.local(loc, true);
    const int64_t rb = A.lrow_begin(), cb = A.lcol_begin();
    spec.m = A.m(); spec.n = A.n(); spec.max_mn = std::max(A.m(), A.n());
    if (target == Target::Devices) {
        internal::Work<double> dsig;
        if (sigma && !sigma->empty()) {
            dsig.resize(Target::Devices, sigma->size());
            hipStream_t st = device::queue(0);
            device::memcpy_async(dsig.data(), sigma->data(), sigma->size() * sizeof(double), st);
            spec.sigma = dsig.data();
        }
        hipStream_t st = device::queue(0);
        slate_amd::dev::generate(spec, lb.m, lb.n, slate_amd::dev::dptr(lb.ptr), lb.ld, s.mb, g.p(), s.rrel(), rb,
                                 A.row0(), s.nb, g.q(), s.crel(), cb, A.col0(), st);
        slate_hip_call(hipStreamSynchronize(st));
        return;
    }
    if (sigma) spec.sigma = sigma->data();
    using R = real_type<T>;
    #pragma omp parallel for schedule(static)
    for (int64_t jl = 0; jl < lb.n; ++jl) {
        int64_t gj = l2g(cb + jl, s.nb, s.crel(), g.q()) - A.col0();
        for (int64_t il = 0; il < lb.m; ++il) {
            int64_t gi = l2g(rb + il, s.mb, s.rrel(), g.p()) - A.row0();
            double re, im;
            gen::entry(spec, gi, gj, is_complex_v<T>, re, im);
            if constexpr (is_complex_v<T>) lb.ptr[il + jl * lb.ld] = T(R(re), R(im));
            else lb.ptr[il + jl * lb.ld] = T(re);
        }
    }
}

/// Diagonal post-op: 'R' make real, 'S' add shift.
template <typename T>
void diag_op(char op, double shift, BaseMatrix<T>& A, Target target) {
    auto& s = *A.storage();
    auto& g = *s.grid;
    Loc loc = internal::loc_of(target);
    LocalBlock<T> lb = A.local(loc, true);
    const int64_t rb = A.lrow_begin(), cb = A.lcol_begin();
    if (target == Target::Devices) {
        hipStream_t st = device::queue(0);
        slate_amd::dev::gen_diag(op, shift, lb.m, lb.n, slate_amd::dev::dptr(lb.ptr), lb.ld, s.mb, g.p(), s.rrel(),
                                 rb, A.row0(), s.nb, g.q(), s.crel(), cb, A.col0(), st);
        slate_hip_call(hipStreamSynchronize(st));
        return;
    }
    for (int64_t jl = 0; jl < lb.n; ++jl) {
        int64_t gj = l2g(cb + jl, s.nb, s.crel(), g.q()) - A.col0();
        for (int64_t il = 0; il < lb.m; ++il) {
            int64_t gi = l2g(rb + il, s.mb, s.rrel(), g.p()) - A.row0();
            if (gi != gj) continue;
            T& a = lb.ptr[il + jl * lb.ld];
            if (op == 'R') a = T(std::real(a));
            else a += T(shift);
        }
    }
}

gen::Spec base_spec(int code, uint64_t seed) {
    gen::Spec sp{};
    sp.code = code;
    sp.seed = seed;
    sp.scale = 1;
    return sp;
}

/// Random orthogonal / unitary Q applied from `side` (Q = Householder QR of
/// a random normal matrix of A's distribution), reference generate_type_svd.hh.
template <typename T>
void apply_random_q(Matrix<T>& A, Side side, Op op, int64_t k, uint64_t seed, Target target, Options const& opts) {
    // U: (side == Left ? m : n) x k, same tiling as A
    int64_t rows = side == Side::Left ? A.m() : A.n();
    Matrix<T> W(std::max(A.m(), A.n()), std::max(A.m(), A.n()), A.mb(), A.nb(), A.grid());
    W.insertLocalTiles(target);
    Matrix<T> U = W.slice(0, rows - 1, 0, k - 1);
    fill(base_spec(gen::Randn, seed), U, target);
    TriangularFactors<T> Tf;
    geqrf(U, Tf, opts);
    unmqr(side, op, U, Tf, A, opts);
}

}  // namespace

std::string generate_matrix_usage() {
    return
        "matrix kind = base[_distribution][_scaling][_modifier]\n"
        "base: zeros ones identity ij jordan jordanT chebspec circul fiedler gfpp kms orthog riemann ris\n"
        "      zielkeNS | rand rands randn randb randr (random) | diag svd poev spd heev syev geev (spectral)\n"
        "distribution (spectral): logrand (default) arith geo cluster0 cluster1 rarith rgeo rcluster0\n"
        "      rcluster1 specified rand rands randn\n"
        "scaling (random, spectral): ufl ofl small large\n"
        "modifier: dominant (random, spectral), zerocolN / zerocolFRAC\n"
        "cond (spectral): requested condition number (default 1/sqrt(eps)); condD: column scaling range\n";
}

template <typename T>
void generate_matrix(MatgenParams& params, Matrix<T>& A, std::vector<real_type<T>>& Sigma, Options const& opts) {
    using R = real_type<T>;
    trace::Block tb("generate_matrix");
    internal::DriverScope ds_;
    Target target = internal::resolve_target(opts);
    Decoded d = decode<R>(params, A.m(), A.n());
    const int64_t m = A.m(), n = A.n(), k = std::min(m, n);
    uint64_t seed = params.seed >= 0 ? uint64_t(params.seed) : uint64_t(std::time(nullptr));
    std::vector<double> S(k, NAN);
    if (d.dist == Dist::Specified) {
        slate_error_if_msg(int64_t(Sigma.size()) != k, "generate_matrix: specified Sigma must have min(m, n) entries");
        for (int64_t i = 0; i < k; ++i) S[i] = double(Sigma[i]);
    }

    if (d.spec == Spectral::None) {
        gen::Spec sp = base_spec(d.code, seed);
        sp.ij_scale = 1.0 / std::pow(10.0, std::ceil(std::log10(double(std::max<int64_t>(n, 1)))));
        if (d.code >= gen::Rand && d.code <= gen::Randr) {
            sp.shift = d.dominant ? double(n) : 0.0;
            sp.scale = d.sigma_max;
        }
        fill(sp, A, target);
        if (d.code == gen::Zeros) std::fill(S.begin(), S.end(), 0.0);
        else if (d.code == gen::Identity) std::fill(S.begin(), S.end(), 1.0);
        else if (d.code == gen::Ones) { std::fill(S.begin(), S.end(), 0.0); if (k) S[0] = std::sqrt(double(m) * n); }
    } else {
        const bool sign = d.spec == Spectral::Heev;
        make_sigma(d, sign, seed, S);
        seed += 1;
        std::vector<double> Sd(S);
        if (d.spec == Spectral::Svd && d.condD != 1) {
            // sum sigma_i^2 = n so the later column scaling keeps the spectrum shape
            double ss = 0;
            for (double v : Sd) ss += v * v;
            const double sc = std::sqrt(double(Sd.size()) / ss);
            for (auto& v : Sd) v *= sc;
        }
        fill(base_spec(gen::Diag, 0), A, target, &Sd);
        if (d.spec == Spectral::Geev && n > 1) {
            // Schur form T: Sigma on the diagonal plus a random strictly upper part
            Matrix<T> Rnd = A.emptyLike();
            Rnd.insertLocalTiles(target);
            // off-diagonal coupling O(1/n) keeps the eigenvalues well conditioned
            gen::Spec up = base_spec(gen::Rands, seed + 11);
            up.scale = 1.0 / double(n);
            fill(up, Rnd, target);
            auto TU = TrapezoidMatrix<T>(Uplo::Upper, Diag::NonUnit, Rnd.slice(0, n - 2, 1, n - 1));
            auto TUp = TrapezoidMatrix<T>(Uplo::Upper, Diag::NonUnit, A.slice(0, n - 2, 1, n - 1));
            add(T(1), TU, T(1), TUp, opts);
        }
        if (d.spec == Spectral::Svd) {
            slate_error_if_msg(m < n, "generate_matrix: svd kind requires m >= n");
            apply_random_q(A, Side::Left, Op::NoTrans, k, seed, target, opts);
            seed += 1;
            apply_random_q(A, Side::Right, Op::ConjTrans, n, seed, target, opts);
            seed += 1;
        } else if (d.spec != Spectral::Diag) {
            // A = Q D Q^H with the same Q on both sides
            Matrix<T> W(n, n, A.mb(), A.nb(), A.grid());
            W.insertLocalTiles(target);
            fill(base_spec(gen::Randn, seed), W, target);
            TriangularFactors<T> Tf;
            geqrf(W, Tf, opts);
            unmqr(Side::Left, Op::NoTrans, W, Tf, A, opts);
            unmqr(Side::Right, Op::ConjTrans, W, Tf, A, opts);
            seed += 1;
            if (d.spec != Spectral::Geev) diag_op('R', 0, A, target);
        }
        if (d.condD != 1 && (d.spec == Spectral::Svd || d.spec == Spectral::Poev || d.spec == Spectral::Heev)) {
            std::vector<R> D(n);
            const double range = std::log(d.condD);
            for (int64_t i = 0; i < n; ++i) D[i] = R(std::exp(gen::rand_sample(gen::Rand, i, 0, seed) * range));
            if (d.spec == Spectral::Svd) scale_row_col(Equed::Col, std::vector<R>{}, D, A, opts);
            else scale_row_col(Equed::Both, D, D, A, opts);
            if (params.verbose) {
                std::printf("D = [");
                for (auto v : D) std::printf(" %11.8g", double(v));
                std::printf(" ];\n");
            }
        }
        if (d.dominant) diag_op('S', double(n), A, target);
    }
    if (d.zero_col >= 0) {
        auto col = A.slice(0, m - 1, d.zero_col, d.zero_col);
        set(T(0), T(0), col, opts);
    }
    Sigma.assign(S.begin(), S.end());
    // Sigma is reported in the matrix's real precision
    for (int64_t i = 0; i < k; ++i) Sigma[i] = R(S[i]);
}

template <typename T>
void generate_matrix(MatgenParams& params, Matrix<T>& A, Options const& opts) {
    std::vector<real_type<T>> S;
    generate_matrix(params, A, S, opts);
}

template <typename T>
void generate_matrix(MatgenParams& params, BaseTrapezoidMatrix<T>& A, std::vector<real_type<T>>& Sigma,
                     Options const& opts) {
    Target target = internal::resolve_target(opts);
    const bool herm = A.matrix_kind() == MatrixKind::Hermitian || A.matrix_kind() == MatrixKind::Symmetric;
    Decoded d = decode<real_type<T>>(params, A.m(), A.n());
    if (d.code == gen::Jordan && A.uplo() == Uplo::Lower)
        bad(params.kind, "jordan matrix is upper triangular; use jordanT for lower");
    if (d.code == gen::JordanT && A.uplo() == Uplo::Upper)
        bad(params.kind, "jordanT matrix is lower triangular; use jordan for upper");
    // generate on the full storage view (both triangles; only the stored one is referenced)
    BaseMatrix<T> base = A;
    base.set_uplo(Uplo::General);
    base.set_kind(MatrixKind::General);
    Matrix<T> G(base);
    MatgenParams p2 = params;
    if (d.zero_col >= 0) {
        // zero row and column of the stored triangle after the fill
        std::string k = params.kind;
        size_t at = k.find("zerocol");
        p2.kind = k.substr(0, at ? at - 1 : 0);
        if (p2.kind.empty()) p2.kind = "rands";
    }
    generate_matrix(p2, G, Sigma, opts);
    params.cond_actual = p2.cond_actual;
    if (herm) diag_op('R', 0, G, target);
    if (d.zero_col >= 0) {
        params.cond_actual = INFINITY;
        auto col = G.slice(0, G.m() - 1, d.zero_col, d.zero_col);
        auto row = G.slice(d.zero_col, d.zero_col, 0, G.n() - 1);
        set(T(0), T(0), col, opts);
        set(T(0), T(0), row, opts);
    }
}

// -----------------------------------------------------------------------------
// Fast grid-independent fill (benchmarks / tests).
template <typename T>
void generate_matrix(std::string const& kind, BaseMatrix<T>& A, uint64_t seed, double shift, Options const& opts) {
    trace::Block tb("generate_matrix");
    internal::DriverScope ds_;
    Target target = internal::resolve_target(opts);
    gen::Spec sp = base_spec(gen::Rands, seed);
    if (shift < 0) shift = double(std::max(A.m(), A.n()));
    if (kind == "spd" || kind == "hpd") { sp.code = gen::SymRands; sp.shift = shift; }
    else if (kind == "diag_dominant" || kind == "rands+n") { sp.code = gen::Rands; sp.shift = shift; }
    else if (kind == "rand_signed") sp.code = gen::Rands;
    else {
        MatgenParams p;
        p.kind = kind;
        Decoded d = decode<real_type<T>>(p, A.m(), A.n());
        slate_error_if_msg(d.spec != Spectral::None || d.zero_col >= 0 || d.dominant || d.sigma_max != 1,
                           "generate_matrix(kind, A): element kinds only; use generate_matrix(MatgenParams, ...)");
        sp.code = d.code;
        sp.ij_scale = 1.0 / std::pow(10.0, std::ceil(std::log10(double(std::max<int64_t>(A.n(), 1)))));
    }
    fill(sp, A, target);
}

#define SLATE_INST_MATGEN(T)                                                                                   \
    template void generate_matrix<T>(MatgenParams&, Matrix<T>&, std::vector<real_type<T>>&, Options const&);    \
    template void generate_matrix<T>(MatgenParams&, Matrix<T>&, Options const&);                               \
    template void generate_matrix<T>(MatgenParams&, BaseTrapezoidMatrix<T>&, std::vector<real_type<T>>&,        \
                                     Options const&);                                                          \
    template void generate_matrix<T>(std::string const&, BaseMatrix<T>&, uint64_t, double, Options const&);
SLATE_INST_MATGEN(float)
SLATE_INST_MATGEN(double)
SLATE_INST_MATGEN(std::complex<float>)
SLATE_INST_MATGEN(std::complex<double>)

}  // namespace slate
