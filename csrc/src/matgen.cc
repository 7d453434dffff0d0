// Test-matrix generation driver (reference matgen/generate_matrix_utils.cc:72-280).
// Host and device share the same counter hash (see kernels/matgen.hip and
// slate_d35_amd/utils/matgen.py), so any grid yields identical matrices.
#include "internal.hh"
#include "slate_amd/matgen.hh"
#include "../kernels/kernels.hh"

namespace slate {

namespace {

inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27; x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}
inline double unit(uint64_t i, uint64_t j, uint64_t seed) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull ^ (j + 0x632BE59BD9B4E019ull) * 0xD1B54A32D192ED03ull
               ^ seed * 0x94D049BB133111EBull;
    return double(mix64(x) >> 11) * (1.0 / 9007199254740992.0);
}

char kind_code(std::string const& k) {
    if (k == "rands" || k == "rand_signed") return 'r';
    if (k == "rand") return 'u';
    if (k == "spd" || k == "poev" || k == "hpd") return 's';
    if (k == "diag_dominant" || k == "rands+n") return 'd';
    if (k == "identity") return 'i';
    if (k == "zeros" || k == "zero") return 'z';
    throw Exception("generate_matrix: unknown kind " + k);
}

}  // namespace

template <typename T>
void generate_matrix(std::string const& kind, BaseMatrix<T>& A, uint64_t seed, double shift, Options const& opts) {
    trace::Block tb("generate_matrix");
    Target target = internal::resolve_target(opts);
    char k = kind_code(kind);
    slate_error_if_msg(A.op() != Op::NoTrans, "generate_matrix: NoTrans view required");
    if ((k == 's' || k == 'd') && shift < 0) shift = double(std::max(A.m(), A.n()));
    auto& s = *A.storage();
    auto& g = *s.grid;
    Loc loc = internal::loc_of(target);
    LocalBlock<T> lbk = A.local(loc, true);
    int64_t rb = A.lrow_begin(), cb = A.lcol_begin();
    if (target == Target::Devices) {
        // shift the local pointer so the kernel's local index 0 is local row rb
        // (the kernel recomputes global indices from absolute local indices)
        T* base = lbk.ptr - rb - cb * lbk.ld;
        hipStream_t st = device::queue(0);
        // generate only the view's block: offset by rb/cb via base + row/col windows
        slate_amd::dev::generate(k, lbk.m, lbk.n, slate_amd::dev::dptr(lbk.ptr), lbk.ld, s.mb, g.p(), s.rrel(),
                                 A.row0() - 0, s.nb, g.q(), s.crel(), A.col0(), seed, shift, st);
        (void)base;
        // local index il of the view block corresponds to absolute local row rb + il
        // -> the kernel treats il as absolute; correct only when rb == 0 and cb == 0
        slate_error_if_msg(rb != 0 || cb != 0, "generate_matrix(device): view must start at the matrix origin");
        slate_hip_call(hipStreamSynchronize(st));
    } else {
        using R = real_type<T>;
        #pragma omp parallel for schedule(static)
        for (int64_t jl = 0; jl < lbk.n; ++jl) {
            int64_t gj = l2g(cb + jl, s.nb, s.crel(), g.q()) - A.col0();
            for (int64_t il = 0; il < lbk.m; ++il) {
                int64_t gi = l2g(rb + il, s.mb, s.rrel(), g.p()) - A.row0();
                uint64_t a = gi, b = gj;
                if (k == 's' && a > b) std::swap(a, b);
                double v;
                if (k == 'i') v = gi == gj ? 1.0 : 0.0;
                else if (k == 'z') v = 0.0;
                else if (k == 'u') v = unit(a, b, seed);
                else v = 2.0 * unit(a, b, seed) - 1.0;
                if ((k == 's' || k == 'd') && gi == gj) v += shift;
                if constexpr (is_complex_v<T>) {
                    double w = (k == 'i' || k == 'z') ? 0.0 : 2.0 * unit(a, b, seed + 7919) - 1.0;
                    if (k == 's') { if (gi == gj) w = 0.0; else if (gi < gj) w = -w; }
                    lbk.ptr[il + jl * lbk.ld] = T(R(v), R(w));
                } else {
                    lbk.ptr[il + jl * lbk.ld] = T(v);
                }
            }
        }
    }
}

template void generate_matrix<float>(std::string const&, BaseMatrix<float>&, uint64_t, double, Options const&);
template void generate_matrix<double>(std::string const&, BaseMatrix<double>&, uint64_t, double, Options const&);
template void generate_matrix<std::complex<float>>(std::string const&, BaseMatrix<std::complex<float>>&, uint64_t, double, Options const&);
template void generate_matrix<std::complex<double>>(std::string const&, BaseMatrix<std::complex<double>>&, uint64_t, double, Options const&);

}  // namespace slate
