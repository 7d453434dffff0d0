// Matrix / vector printing (reference include/slate/print.hh, src/print.cc).
//
// Output is MATLAB/Octave-style `label = [ ... ];` on rank 0, so it can be
// pasted back into a script.  Option::PrintVerbose:
//   0 nothing; 1 metadata (dims, tiling, grid, kind); 2 metadata + the first
//   and last PrintEdgeItems rows/columns with "..." between them (the
//   default); 3 same as 2 but every tile's corner; 4 the whole matrix.
// Only the printed parts are gathered (corner slices), not the whole matrix.
// For triangular/symmetric/Hermitian/band kinds the entries outside the
// stored part print as 0 (unit diagonals as 1).
#include "internal.hh"

#include <cstdio>
#include <sstream>

namespace slate {

using namespace internal;

template <typename R>
int snprintf_value(char* buf, size_t len, int width, int precision, R v) {
    if constexpr (std::is_integral_v<R>) return std::snprintf(buf, len, " %*lld", width, (long long)v);
    else if (v == R(0)) return std::snprintf(buf, len, " %*.0f%*s", width - precision, 0.0, precision, "");
    else return std::snprintf(buf, len, " %*.*f", width, precision, double(v));
}

template <typename R>
int snprintf_value(char* buf, size_t len, int width, int precision, std::complex<R> v) {
    int n = snprintf_value(buf, len, width, precision, v.real());
    n += std::snprintf(buf + n, len - size_t(n), " + ");
    n += snprintf_value(buf + n, len - size_t(n), width, precision, v.imag());
    n += std::snprintf(buf + n, len - size_t(n), "i");
    return n;
}

namespace {

struct PrintOpts {
    int verbose, edge, width, precision;
};

PrintOpts print_opts(Options const& opts) {
    return {int(get_option<int64_t>(opts, Option::PrintVerbose, 2)), int(get_option<int64_t>(opts, Option::PrintEdgeItems, 16)),
            int(get_option<int64_t>(opts, Option::PrintWidth, 10)), int(get_option<int64_t>(opts, Option::PrintPrecision, 4))};
}

const char* kind_name(MatrixKind k) {
    switch (k) {
        case MatrixKind::General: return "general";
        case MatrixKind::Trapezoid: return "trapezoid";
        case MatrixKind::Triangular: return "triangular";
        case MatrixKind::Symmetric: return "symmetric";
        case MatrixKind::Hermitian: return "Hermitian";
        case MatrixKind::Band: return "band";
        case MatrixKind::TriangularBand: return "triangular band";
        case MatrixKind::HermitianBand: return "Hermitian band";
    }
    return "?";
}

/// value of logical (i, j) as the matrix kind defines it
template <typename T>
T masked(BaseMatrix<T> const& A, int64_t i, int64_t j, T v) {
    Uplo u = A.uplo();
    if ((u == Uplo::Lower && j > i) || (u == Uplo::Upper && i > j)) return T(0);
    if (A.kl() || A.ku() || A.matrix_kind() == MatrixKind::Band) {
        if (i - j > A.kl() || j - i > A.ku()) return T(0);
    }
    if (i == j && A.diag() == Diag::Unit) return T(1);
    return v;
}

/// gathered dense copy of rows [r0, r1) x cols [c0, c1) of A (logical)
template <typename T>
std::vector<T> corner(BaseMatrix<T> const& A, int64_t r0, int64_t r1, int64_t c0, int64_t c1, Options const& opts) {
    std::vector<T> h;
    if (r1 <= r0 || c1 <= c0) return h;
    BaseMatrix<T> S = A.slice(r0, r1 - 1, c0, c1 - 1);
    gather(S, h, opts);
    for (int64_t j = c0; j < c1; ++j)
        for (int64_t i = r0; i < r1; ++i) {
            T& v = h[(i - r0) + (j - c0) * (r1 - r0)];
            v = masked(A, i, j, v);
        }
    return h;
}

template <typename T>
std::string print_impl(const char* label, BaseMatrix<T> const& A, Options const& opts) {
    PrintOpts po = print_opts(opts);
    if (po.verbose <= 0) return "";
    auto g = A.grid();
    const bool root = g->rank() == 0;
    const int64_t m = A.m(), n = A.n();
    std::ostringstream out;
    if (root) {
        out << "% " << label << ": " << m << "-by-" << n << ", " << A.mt() << "-by-" << A.nt() << " tiles, tileSize "
            << A.mb() << "-by-" << A.nb() << ", " << kind_name(A.matrix_kind());
        if (A.uplo() != Uplo::General) out << " uplo " << char(A.uplo());
        if (A.op() != Op::NoTrans) out << " op " << char(A.op());
        if (A.kl() || A.ku()) out << " kl " << A.kl() << " ku " << A.ku();
        out << ", grid " << g->p() << "x" << g->q() << "\n";
    }
    if (po.verbose == 1) return out.str();
    // row / column index sets to print
    auto pick = [&](int64_t dim, int64_t tsize, std::vector<std::pair<int64_t, int64_t>>& ranges) {
        if (po.verbose >= 4 || dim <= 2 * po.edge) { ranges.push_back({0, dim}); return; }
        if (po.verbose == 3) {
            // first and last edge/2 of every tile
            int64_t e = std::max(1, po.edge / 2);
            for (int64_t t0 = 0; t0 < dim; t0 += tsize) {
                int64_t t1 = std::min(dim, t0 + tsize);
                if (t1 - t0 <= 2 * e) ranges.push_back({t0, t1});
                else { ranges.push_back({t0, t0 + e}); ranges.push_back({t1 - e, t1}); }
            }
            return;
        }
        ranges.push_back({0, po.edge});
        ranges.push_back({dim - po.edge, dim});
    };
    std::vector<std::pair<int64_t, int64_t>> rr, cr;
    pick(m, A.mb(), rr);
    pick(n, A.nb(), cr);
    char buf[128];
    if (root) out << label << " = [\n";
    for (size_t a = 0; a < rr.size(); ++a) {
        std::vector<std::vector<T>> blocks;
        for (auto& c : cr) blocks.push_back(corner(A, rr[a].first, rr[a].second, c.first, c.second, opts));
        if (!root) continue;
        if (a > 0 && rr[a].first != rr[a - 1].second) out << "  ...\n";
        const int64_t nr = rr[a].second - rr[a].first;
        for (int64_t i = 0; i < nr; ++i) {
            for (size_t b = 0; b < cr.size(); ++b) {
                if (b > 0 && cr[b].first != cr[b - 1].second) out << "  ...";
                const int64_t nc = cr[b].second - cr[b].first;
                for (int64_t j = 0; j < nc; ++j) {
                    snprintf_value(buf, sizeof(buf), po.width, po.precision, blocks[b][i + j * nr]);
                    out << buf;
                }
            }
            out << "\n";
        }
    }
    if (root) out << "];\n";
    return out.str();
}

}  // namespace

template <typename T>
void print(const char* label, BaseMatrix<T> const& A, Options const& opts) {
    std::string s = print_impl(label, A, opts);
    if (!s.empty()) {
        std::fputs(s.c_str(), stdout);
        std::fflush(stdout);
    }
}

template <typename T>
void print(const char* label, int64_t n, T const* x, int64_t incx, Options const& opts) {
    PrintOpts po = print_opts(opts);
    if (po.verbose <= 0 || default_grid()->rank() != 0) return;
    std::ostringstream out;
    char buf[128];
    out << label << " = [";
    const bool cut = po.verbose < 4 && n > 2 * po.edge;
    for (int64_t i = 0; i < n; ++i) {
        if (cut && i == po.edge) { out << "  ..."; i = n - po.edge; }
        snprintf_value(buf, sizeof(buf), po.width, po.precision, x[i * incx]);
        out << buf;
    }
    out << " ];\n";
    std::fputs(out.str().c_str(), stdout);
    std::fflush(stdout);
}

template <typename T>
std::string print_to_string(const char* label, BaseMatrix<T> const& A, Options const& opts) {
    return print_impl(label, A, opts);
}

#define SLATE_PRINT_INST(T)                                                                     \
    template void print<T>(const char*, BaseMatrix<T> const&, Options const&);                  \
    template void print<T>(const char*, int64_t, T const*, int64_t, Options const&);            \
    template std::string print_to_string<T>(const char*, BaseMatrix<T> const&, Options const&);

SLATE_PRINT_INST(float)
SLATE_PRINT_INST(double)
SLATE_PRINT_INST(std::complex<float>)
SLATE_PRINT_INST(std::complex<double>)
template void print<int64_t>(const char*, int64_t, int64_t const*, int64_t, Options const&);

}  // namespace slate
