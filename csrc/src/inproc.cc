// In-process ranks (see inproc.hh).
#include "slate_amd/inproc.hh"
#include "internal.hh"

#include <atomic>
#include <cmath>
#include <cstring>
#include <exception>
#include <mutex>
#include <map>
#include <thread>
#include <tuple>

namespace slate {

namespace {
std::mutex g_run_mtx;
// device contexts of the rank threads, reused across runs (stream creation
// and the allocator's cache survive from one LAPACK call to the next)
std::vector<device::Context*> g_ctx;
std::vector<int> g_ctx_dev;
std::atomic<int64_t> g_runs{0};
int g_last_p = 0, g_last_q = 0;
}  // namespace

int64_t inproc_run_count() { return g_runs.load(); }

namespace { thread_local bool t_in_rank = false; }
bool in_inproc_rank() { return t_in_rank; }
void inproc_last_shape(int& p, int& q) { p = g_last_p; q = g_last_q; }

bool multi_process_job() {
    auto num = [](const char* k) { const char* e = std::getenv(k); return e ? std::atoi(e) : 0; };
    return num("WORLD_SIZE") > 1 || std::getenv("LOCAL_RANK") || num("OMPI_COMM_WORLD_SIZE") > 1 ||
           num("PMI_SIZE") > 1 || num("PMIX_SIZE") > 1 || (std::getenv("SLURM_PROCID") && num("SLURM_NTASKS") > 1);
}

int inproc_ranks() {
    if (const char* e = std::getenv("SLATE_INPROC_RANKS")) return std::max(1, std::atoi(e));
    if (!device::available()) return 1;
    // One process per GPU (torchrun / MPI environment, a p x q grid already
    // set up, or a program that picked its device): stay on this process's
    // GPU -- spreading every process over all GPUs would oversubscribe them.
    if (multi_process_job() || device::device_explicit()) return 1;
    if (auto g = default_grid(); g && g->size() > 1) return 1;
    return std::max(1, device::count());
}

void inproc_grid_shape(int n, int& p, int& q) {
    p = int(std::sqrt(double(n)));
    while (p > 1 && n % p) --p;
    q = n / p;
}

namespace {
std::atomic<int64_t> g_copy_bytes{0};
std::mutex g_groups_mtx;
std::map<std::tuple<int, int, int, std::vector<int>>, std::shared_ptr<InprocGroup>>& groups() {
    static auto* m = new std::map<std::tuple<int, int, int, std::vector<int>>, std::shared_ptr<InprocGroup>>();
    return *m;
}
}  // namespace

int64_t inproc_copy_bytes() { return g_copy_bytes.load(); }

InprocGroup::InprocGroup(int p, int q, GridOrder order, std::vector<int> devices)
    : p_(p), q_(q), order_(order), devices_(std::move(devices)) {
    grids_ = make_thread_grids(p, q, order, devices_);
}

std::shared_ptr<InprocGroup> InprocGroup::get(int p, int q, std::vector<int> devices, GridOrder order) {
    slate_error_if_msg(p < 1 || q < 1, "InprocGroup: p, q >= 1");
    const int n = p * q;
    const bool dev = device::available();
    if (dev && devices.empty())
        for (int r = 0; r < n; ++r) devices.push_back(r % device::count());
    if (!dev) devices.clear();
    slate_error_if_msg(dev && int(devices.size()) != n, "InprocGroup: one device per rank");
    std::lock_guard<std::mutex> l(g_groups_mtx);
    auto key = std::make_tuple(p, q, int(order), devices);
    auto& slot = groups()[key];
    if (!slot) slot = std::make_shared<InprocGroup>(p, q, order, devices);
    return slot;
}

std::shared_ptr<InprocGroup> InprocGroup::of_size(int n) {
    if (n <= 0) n = inproc_ranks();
    int p, q;
    inproc_grid_shape(n, p, q);
    return get(p, q);
}

void InprocGroup::run(std::function<void(int, GridPtr const&)> const& fn) {
    std::lock_guard<std::mutex> run_lock(g_run_mtx);
    const int n = size();
    ++g_runs;
    g_last_p = p_;
    g_last_q = q_;
    const bool dev = !devices_.empty();
    if (dev) {
        if (int(g_ctx.size()) < n) { g_ctx.resize(n, nullptr); g_ctx_dev.resize(n, -1); }
        for (int r = 0; r < n; ++r)
            if (!g_ctx[r] || g_ctx_dev[r] != devices_[r]) {
                if (g_ctx[r]) device::context_destroy(g_ctx[r]);
                g_ctx[r] = device::context_create(devices_[r]);
                g_ctx_dev[r] = devices_[r];
            }
    }
    std::vector<std::exception_ptr> err(n);
    std::vector<std::thread> th;
    for (int r = 0; r < n; ++r) {
        th.emplace_back([&, r] {
            t_in_rank = true;
            try {
                if (dev) device::context_bind(g_ctx[r]);
                set_thread_default_grid(grids_[r]);
                fn(r, grids_[r]);
                if (dev) device::sync_all();
            } catch (...) {
                err[r] = std::current_exception();
                thread_grid_abort(*grids_[r]);   // wake the ranks waiting on me
            }
            set_thread_default_grid(nullptr);
            if (dev) {
                try { device::sync_all(); } catch (...) {}
                device::context_bind(nullptr);
            }
        });
    }
    for (auto& t : th) t.join();
    // report the root cause: a rank that failed on its own, not one woken by an abort
    std::exception_ptr first;
    for (auto& e : err) {
        if (!e) continue;
        try { std::rethrow_exception(e); }
        catch (CommException const&) { if (!first) first = e; continue; }
        catch (...) { first = e; break; }
    }
    if (first) {
        for (auto& g : grids_) thread_grid_reset(*g);   // the group stays usable
        std::rethrow_exception(first);
    }
}

void run_in_process(int p, int q, std::function<void(int, GridPtr const&)> const& fn, std::vector<int> devices,
                    GridOrder order) {
    InprocGroup::get(p, q, std::move(devices), order)->run(fn);
}

template <typename T>
void scatter_from_host(T const* A, int64_t lda, Matrix<T>& M, Target target) {
    using namespace internal;
    const Loc loc = loc_of(target);
    LocalBlock<T> L = M.local(loc, true);
    if (L.empty()) return;
    auto& g = *M.grid();
    hipStream_t s = target == Target::Devices ? device::queue(device::kCommQueue) : nullptr;
    for (int64_t j = 0; j < M.nt(); ++j) {
        if (M.scol_owner(j) != g.mycol()) continue;
        const int64_t lc = lcol_of(M, j), gc = gcol_of(M, j), nbj = M.tileNb(j);
        for (int64_t i = 0; i < M.mt(); ++i) {
            if (M.srow_owner(i) != g.myrow()) continue;
            const int64_t lr = lrow_of(M, i), gr = grow_of(M, i), mbi = M.tileMb(i);
            T const* src = A + gr + gc * lda;
            T* dst = L.ptr + lr + lc * L.ld;
            g_copy_bytes += mbi * nbj * int64_t(sizeof(T));
            if (s) device::memcpy2d_async(dst, L.ld * sizeof(T), src, lda * sizeof(T), mbi * sizeof(T), nbj, s);
            else for (int64_t c = 0; c < nbj; ++c) std::memcpy(dst + c * L.ld, src + c * lda, mbi * sizeof(T));
        }
    }
    if (s) slate_hip_call(hipStreamSynchronize(s));
}

template <typename T>
void gather_to_host(Matrix<T>& M, T* A, int64_t lda) {
    using namespace internal;
    auto& st = *M.storage();
    const bool on_dev = st.has(Loc::Device) && st.state(Loc::Device) != Invalid;
    const Loc loc = on_dev ? Loc::Device : Loc::Host;
    LocalBlock<T> L = M.local(loc, false);
    if (L.empty()) return;
    auto& g = *M.grid();
    hipStream_t s = loc == Loc::Device ? device::queue(device::kCommQueue) : nullptr;
    if (s) device::sync_all();
    for (int64_t j = 0; j < M.nt(); ++j) {
        if (M.scol_owner(j) != g.mycol()) continue;
        const int64_t lc = lcol_of(M, j), gc = gcol_of(M, j), nbj = M.tileNb(j);
        for (int64_t i = 0; i < M.mt(); ++i) {
            if (M.srow_owner(i) != g.myrow()) continue;
            const int64_t lr = lrow_of(M, i), gr = grow_of(M, i), mbi = M.tileMb(i);
            T const* src = L.ptr + lr + lc * L.ld;
            T* dst = A + gr + gc * lda;
            g_copy_bytes += mbi * nbj * int64_t(sizeof(T));
            if (s) device::memcpy2d_async(dst, lda * sizeof(T), src, L.ld * sizeof(T), mbi * sizeof(T), nbj, s);
            else for (int64_t c = 0; c < nbj; ++c) std::memcpy(dst + c * lda, src + c * L.ld, mbi * sizeof(T));
        }
    }
    if (s) slate_hip_call(hipStreamSynchronize(s));
}

#define SLATE_INPROC_INST(T)                                                          \
    template void scatter_from_host<T>(T const*, int64_t, Matrix<T>&, Target);      \
    template void gather_to_host<T>(Matrix<T>&, T*, int64_t);

SLATE_INPROC_INST(float)
SLATE_INPROC_INST(double)
SLATE_INPROC_INST(std::complex<float>)
SLATE_INPROC_INST(std::complex<double>)

}  // namespace slate
