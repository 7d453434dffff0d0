// Debug utilities (reference src/auxiliary/Debug.cc): see debug.hh for how
// the per-tile checks map onto per-process local arrays.
#include "slate_amd/debug.hh"
#include "slate_amd/device.hh"

#include <atomic>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <sstream>

namespace slate {

namespace {

std::atomic<int>& flag() {
    static std::atomic<int> f{[] {
        const char* e = std::getenv("SLATE_DEBUG");
        return (e && std::atoi(e) != 0) ? 1 : 0;
    }()};
    return f;
}

char mosi_letter(MOSI_State st, bool present) {
    if (!present) return '-';
    char c = (st & Modified) ? 'M' : (st & Shared) ? 'S' : 'I';
    if (st & OnHold) c = char(c + ('a' - 'A'));   // on hold: lower case
    return c;
}

template <typename T>
double absval(T v) { return std::abs(v); }

}  // namespace

void Debug::on() { flag() = 1; }
void Debug::off() { flag() = 0; }
bool Debug::enabled() { return flag() != 0; }

template <typename T>
int64_t Debug::diffLapackMatrices(int64_t m, int64_t n, T const* A, int64_t lda, T const* B, int64_t ldb,
                                  int64_t mb, int64_t nb, double tol, std::string* out) {
    slate_error_if_msg(mb <= 0 || nb <= 0, "diffLapackMatrices: tile sizes must be positive");
    double amax = 0;
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < m; ++i) amax = std::max(amax, absval(A[i + j * lda]));
    const double thresh = tol * amax;
    std::ostringstream os;
    int64_t ndiff = 0;
    for (int64_t i0 = 0; i0 < m; i0 += mb) {
        for (int64_t j0 = 0; j0 < n; j0 += nb) {
            bool same = true;
            for (int64_t j = j0; j < std::min(n, j0 + nb) && same; ++j)
                for (int64_t i = i0; i < std::min(m, i0 + mb); ++i)
                    if (absval(A[i + j * lda] - B[i + j * ldb]) > thresh) { same = false; break; }
            os << (same ? '.' : '#');
            ndiff += !same;
        }
        os << '\n';
    }
    if (out) *out = os.str();
    if (enabled()) std::cout << os.str() << std::flush;
    return ndiff;
}

template <typename T>
int64_t Debug::checkTilesLives(BaseMatrix<T> const& A) {
    auto s = A.storage();
    const bool any_local = s->mloc > 0 && s->nloc > 0;
    int64_t bad = 0;
    bool backed = false;
    for (Loc loc : {Loc::Host, Loc::Device})
        if (s->has(loc) && s->state(loc) != Invalid) backed = true;
    if (!any_local) return 0;
    for (int64_t j = 0; j < A.nt(); ++j)
        for (int64_t i = 0; i < A.mt(); ++i)
            if (A.tileIsLocal(i, j) && !backed) ++bad;
    if (bad && enabled())
        std::cout << "[rank " << A.mpiRank() << "] checkTilesLives: " << bad
                  << " local tiles without a live valid instance\n" << std::flush;
    return bad;
}

template <typename T>
bool Debug::checkTilesLayout(BaseMatrix<T> const& A) {
    auto s = A.storage();
    bool ok = true;
    for (Loc loc : {Loc::Host, Loc::Device}) {
        if (!s->has(loc)) continue;
        // local arrays are column-major by construction; the leading
        // dimension must cover the local rows
        if (s->ld(loc) < std::max<int64_t>(1, s->mloc)) ok = false;
    }
    if (!ok && enabled())
        std::cout << "[rank " << A.mpiRank() << "] checkTilesLayout: ld smaller than local rows\n" << std::flush;
    return ok;
}

template <typename T>
std::string Debug::printTiles(BaseMatrix<T> const& A) {
    auto s = A.storage();
    std::ostringstream os;
    const int me = A.mpiRank();
    const char hs = mosi_letter(s->state(Loc::Host), s->has(Loc::Host));
    const char ds = mosi_letter(s->state(Loc::Device), s->has(Loc::Device));
    os << "[rank " << me << "] " << A.m() << " x " << A.n() << " matrix, " << A.mt() << " x " << A.nt()
       << " tiles, origin " << (s->origin() == Loc::Host ? "host" : "device")
       << ", kind " << char(s->kind()) << "; tile = owner:host/device MOSI ('-' no instance, '..' remote)\n";
    for (int64_t i = 0; i < A.mt(); ++i) {
        for (int64_t j = 0; j < A.nt(); ++j) {
            int r = A.tileRank(i, j);
            char buf[32];
            if (r == me) std::snprintf(buf, sizeof(buf), " %3d:%c%c", r, hs, ds);
            else std::snprintf(buf, sizeof(buf), " %3d:..", r);
            os << buf;
        }
        os << '\n';
    }
    if (enabled()) std::cout << os.str() << std::flush;
    return os.str();
}

std::string Debug::printNumFreeMemBlocks() {
    std::ostringstream os;
    if (!device::available()) {
        os << "device allocator: no device\n";
    } else {
        os << "device allocator: " << device::blocks_in_use() << " blocks / " << device::bytes_in_use()
           << " bytes in use, " << device::blocks_cached() << " blocks / " << device::bytes_cached()
           << " bytes cached; pinned host " << device::host_bytes_in_use() << " bytes\n";
    }
    if (enabled()) std::cout << os.str() << std::flush;
    return os.str();
}

size_t Debug::checkDeviceMemoryLeaks() {
    size_t b = device::available() ? device::bytes_in_use() : 0;
    if (b && enabled()) std::cout << "checkDeviceMemoryLeaks: " << b << " bytes still in use\n" << std::flush;
    return b;
}

size_t Debug::checkHostMemoryLeaks() {
    size_t b = device::available() ? device::host_bytes_in_use() : 0;
    if (b && enabled()) std::cout << "checkHostMemoryLeaks: " << b << " pinned bytes still in use\n" << std::flush;
    return b;
}

#define SLATE_DEBUG_INST(T)                                                                                   \
    template int64_t Debug::diffLapackMatrices<T>(int64_t, int64_t, T const*, int64_t, T const*, int64_t,    \
                                                  int64_t, int64_t, double, std::string*);                   \
    template int64_t Debug::checkTilesLives<T>(BaseMatrix<T> const&);                                        \
    template bool Debug::checkTilesLayout<T>(BaseMatrix<T> const&);                                          \
    template std::string Debug::printTiles<T>(BaseMatrix<T> const&);
SLATE_DEBUG_INST(float)
SLATE_DEBUG_INST(double)
SLATE_DEBUG_INST(std::complex<float>)
SLATE_DEBUG_INST(std::complex<double>)
#undef SLATE_DEBUG_INST

}  // namespace slate
