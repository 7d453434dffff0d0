// Device runtime implementation (see device.hh).
#include "slate_amd/device.hh"

#include <cstdlib>
#include <algorithm>
#include <atomic>
#include <deque>
#include <string>

namespace slate {

bool multi_process_job();   // inproc.cc: a launcher started one process per GPU

namespace device {

namespace {

// bumped whenever a block goes back to HIP (hipFree): address-keyed caches
// of other subsystems (IPC handles of the peer broadcast) use it to notice
// that an address may now name a different allocation
std::atomic<uint64_t> g_free_epoch{0};

struct State {
    std::mutex mtx;
    int device = -1;
    bool streams_ready = false;
    bool destroyed = false;   // context_destroy ran while blocks were still live
    int reserved_cus = 0;
    int full_queue = 0;        // a queue whose kernels may use every CU
    hipStream_t streams[kNumQueues] = {};
    std::vector<hipEvent_t> events;
    // caching allocator: bucket size -> free list; ptr -> bucket size
    std::multimap<size_t, void*> free_blocks;
    std::map<void*, size_t> live;
    size_t in_use = 0, cached = 0;
    // stream-ordered frees: a freed block is reusable once the work queued
    // before the free on every queue (and the null stream) has drained
    struct Pending { void* p; size_t b; std::vector<hipEvent_t> ev; };
    std::deque<Pending> pending;
    // stream-private free lists (free_async): a block freed on stream s is
    // reused at once by the next malloc_async on s -- stream order makes that
    // safe without waiting for an event
    std::map<hipStream_t, std::multimap<size_t, void*>> stream_free;
    std::map<void*, hipStream_t> live_stream;      // blocks from malloc_async
    size_t stream_cached = 0;
    std::map<void*, size_t> host_live;   // pinned host blocks
    size_t host_in_use = 0;
};

void flush_stream_free_locked(State& s);

State& process_state() {
    static State* s = new State();  // intentionally leaked: outlives static dtors
    return *s;
}

// the calling thread's bound context (nullptr: the process context)
thread_local State* t_ctx = nullptr;

State& st() { return t_ctx ? *t_ctx : process_state(); }

// owner of every device block, so a block freed by another thread (e.g. a
// matrix made by a rank thread and dropped by the main thread) returns to the
// context that allocated it
std::mutex g_owner_mtx;
std::map<void*, State*>& owners() {
    static auto* m = new std::map<void*, State*>();
    return *m;
}
bool g_multi_ctx = false;   // any context besides the process one ever made

void own(void* p, State* s) {
    if (!g_multi_ctx) return;
    std::lock_guard<std::mutex> l(g_owner_mtx);
    owners()[p] = s;
}
State& owner_of(void* p) {
    if (!g_multi_ctx) return st();
    std::lock_guard<std::mutex> l(g_owner_mtx);
    auto it = owners().find(p);
    if (it == owners().end()) {
        // allocated by the process context before any other context existed
        // (so never recorded): return it there, not to the freeing thread's
        State& ps = process_state();
        std::lock_guard<std::mutex> g(ps.mtx);
        return ps.live.count(p) ? ps : st();
    }
    State* s = it->second;
    owners().erase(it);
    return *s;
}

size_t bucket(size_t bytes) {
    // round to 2 MiB for large blocks, power-of-two-ish for small ones
    const size_t big = size_t(2) << 20;
    if (bytes >= big) return (bytes + big - 1) / big * big;
    size_t b = 256;
    while (b < bytes) b <<= 1;
    return b;
}

void ensure_device_locked(State& s) {
    if (s.device >= 0) return;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        throw DeviceException("no HIP device available", __func__, __FILE__, __LINE__);
    int dev = 0;
    if (const char* lr = std::getenv("LOCAL_RANK")) dev = std::atoi(lr) % n;
    slate_hip_call(hipSetDevice(dev));
    s.device = dev;
}

void ensure_streams_locked(State& s) {
    ensure_device_locked(s);
    if (s.streams_ready) return;
    int lo = 0, hi = 0;
    slate_hip_call(hipDeviceGetStreamPriorityRange(&lo, &hi));
    // CU partitioning (SLATE_PANEL_CUS=R, 0 = off): the trailing-update queue
    // (and by default the lookahead queue) run on a CU mask that leaves R CUs
    // free, so the panel chain's short kernels always find idle CUs instead of
    // waiting for a SIMD of the trailing GEMM to drain.
    //
    // Mask bit i selects a CU of XCC (i mod #XCC) -- the KFD deals user-mask
    // bits round-robin over the XCCs -- so reserving bits 0 .. R-1 takes R/8
    // CUs from every XCD and the XCD-balanced trailing GEMM loses R/256 of its
    // rate (round 5 reserved bits c % (256/R) == 0, i.e. all of them on XCD 0,
    // which then ran the balanced GEMM at the speed of a crippled XCD; the
    // placement and the complement-mask GEMM rate are measured by
    // csrc/tools/cu_mask_probe.hip, profiles/r6_cu_mask_probe.txt).
    //
    // SLATE_PANEL_CUS_MODE: "shared" (default) keeps the panel and comm queues
    // unmasked at high priority -- they may use every CU, and the R reserved
    // ones are never held by the update; "exclusive" confines them to the R
    // reserved CUs (a masked stream cannot carry a priority).
    // SLATE_PANEL_CUS_LA=0 leaves the lookahead queue unmasked as well.
    int ncu = 0, nxcc = 1;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, s.device) == hipSuccess) ncu = prop.multiProcessorCount;
        int x = 0;
        if (hipDeviceGetAttribute(&x, hipDeviceAttributeNumberOfXccs, s.device) == hipSuccess && x > 0) nxcc = x;
    }
    // default: 32 CUs (one per shader engine, so the SE-balanced dispatcher
    // loses exactly 1/8) for one-process-per-GPU jobs, whose p x q panel
    // chains are longer than their trailing updates; 0 on one GPU, where the
    // update dominates (profiles/r6_cu_mask_bench_ab.txt: -9 %), and for
    // in-process ranks.  The 2 x 4 critical-path model:
    // profiles/r6_critpath_2x4_cus_nonblocking.txt.
    int reserve = multi_process_job() ? 32 : 0;
    if (const char* e = std::getenv("SLATE_PANEL_CUS")) reserve = std::atoi(e);
    if (ncu < 64) reserve = 0;
    reserve = std::max(0, std::min(reserve, ncu / 2));
    reserve = (reserve + nxcc - 1) / nxcc * nxcc;   // whole CUs per XCC
    bool exclusive = false, mask_la = true;
    if (const char* e = std::getenv("SLATE_PANEL_CUS_MODE")) exclusive = std::string(e) == "exclusive";
    if (const char* e = std::getenv("SLATE_PANEL_CUS_LA")) mask_la = std::atoi(e) != 0;
    std::vector<uint32_t> mask_panel, mask_update;
    if (reserve > 0) {
        const int words = (ncu + 31) / 32;
        mask_panel.assign(words, 0);
        mask_update.assign(words, 0);
        for (int c = 0; c < ncu; ++c)
            (c < reserve ? mask_panel : mask_update)[c / 32] |= (1u << (c % 32));
    }
    s.reserved_cus = reserve;
    s.full_queue = (reserve > 0 && !exclusive) ? 1 : (reserve > 0 ? kCommQueue : 0);
    for (int i = 0; i < kNumQueues; ++i) {
        const bool panel = (i == 1 || i == kCommQueue);
        const bool masked = reserve > 0 &&
            (panel ? exclusive : (i == kTrailQueue || (i == kLookaheadQueue && mask_la)));
        if (masked) {
            auto& m = panel ? mask_panel : mask_update;
            slate_hip_call(hipExtStreamCreateWithCUMask(&s.streams[i], uint32_t(m.size() * 32), m.data()));
        } else {
            const int prio = panel ? hi : lo;
            slate_hip_call(hipStreamCreateWithPriority(&s.streams[i], hipStreamNonBlocking, prio));
        }
    }
    s.streams_ready = true;
}

hipEvent_t event_get_locked(State& s) {
    if (!s.events.empty()) {
        hipEvent_t e = s.events.back();
        s.events.pop_back();
        return e;
    }
    hipEvent_t e;
    slate_hip_call(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
}

/// move pending frees whose events have completed to the free lists
/// (wait: block until all of them have)
void reclaim_locked(State& s, bool wait) {
    for (auto it = s.pending.begin(); it != s.pending.end();) {
        bool done = true;
        for (hipEvent_t e : it->ev) {
            if (wait) { slate_hip_call(hipEventSynchronize(e)); continue; }
            hipError_t r = hipEventQuery(e);
            if (r == hipErrorNotReady) { done = false; break; }
            slate_hip_call(r);
        }
        if (!done) { ++it; continue; }
        for (hipEvent_t e : it->ev) s.events.push_back(e);
        s.free_blocks.emplace(it->b, it->p);
        s.cached += it->b;
        it = s.pending.erase(it);
    }
}

}  // namespace

struct Context : State {};

Context* context_create(int dev) {
    int n = count();
    slate_error_if_msg(n <= 0, "context_create: no HIP device");
    slate_error_if_msg(dev < 0 || dev >= n, "context_create: device out of range");
    g_multi_ctx = true;
    auto* c = new Context();
    c->device = dev;
    return c;
}

void context_bind(Context* ctx) {
    t_ctx = ctx;
    if (ctx) slate_hip_call(hipSetDevice(ctx->device));
    else if (process_state().device >= 0) slate_hip_call(hipSetDevice(process_state().device));
}

Context* context_current() { return static_cast<Context*>(t_ctx); }

int context_device(Context* ctx) { return ctx ? ctx->device : get_device(); }

void context_destroy(Context* ctx) {
    if (!ctx) return;
    State* prev = t_ctx;
    t_ctx = ctx;
    (void)hipSetDevice(ctx->device);
    {
        std::lock_guard<std::mutex> g(ctx->mtx);
        if (ctx->streams_ready)
            for (int i = 0; i < kNumQueues; ++i) (void)hipStreamSynchronize(ctx->streams[i]);
        reclaim_locked(*ctx, true);
        flush_stream_free_locked(*ctx);
        for (auto& kv : ctx->free_blocks) (void)hipFree(kv.second);
        ++g_free_epoch;
        ctx->free_blocks.clear();
        ctx->cached = 0;
        for (auto e : ctx->events) (void)hipEventDestroy(e);
        ctx->events.clear();
        if (ctx->streams_ready)
            for (int i = 0; i < kNumQueues; ++i) (void)hipStreamDestroy(ctx->streams[i]);
        ctx->streams_ready = false;
    }
    t_ctx = prev;
    context_bind(static_cast<Context*>(prev));
    // blocks still live (handed out, not yet freed) keep the context alive;
    // free() deletes it with its last block
    bool empty;
    {
        std::lock_guard<std::mutex> g(ctx->mtx);
        empty = ctx->live.empty();
        ctx->destroyed = !empty;
    }
    if (empty) delete ctx;
}

int reserved_cus() { return st().reserved_cus; }

int full_queue() {
    auto& s = st();
    std::lock_guard<std::mutex> g(s.mtx);
    ensure_streams_locked(s);
    return s.full_queue;
}

bool available() {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess && n > 0;
}

int count() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

namespace { std::atomic<bool> g_explicit_device{false}; }
uint64_t alloc_epoch() { return g_free_epoch.load(); }
bool device_explicit() { return g_explicit_device.load(); }

void set_device(int dev) {
    auto& s = st();
    std::lock_guard<std::mutex> g(s.mtx);
    g_explicit_device = true;
    if (s.device == dev) return;
    slate_error_if_msg(s.streams_ready, "set_device after streams were created");
    slate_hip_call(hipSetDevice(dev));
    s.device = dev;
}

int get_device() {
    auto& s = st();
    std::lock_guard<std::mutex> g(s.mtx);
    ensure_device_locked(s);
    return s.device;
}

hipStream_t queue(int index) {
    auto& s = st();
    std::lock_guard<std::mutex> g(s.mtx);
    ensure_streams_locked(s);
    slate_assert(index >= 0 && index < kNumQueues);
    return s.streams[index];
}

void sync_all() {
    auto& s = st();
    if (!s.streams_ready) return;
    for (int i = 0; i < kNumQueues; ++i)
        slate_hip_call(hipStreamSynchronize(s.streams[i]));
}

hipEvent_t event_get() {
    auto& s = st();
    std::lock_guard<std::mutex> g(s.mtx);
    ensure_device_locked(s);
    return event_get_locked(s);
}

void event_put(hipEvent_t e) {
    auto& s = st();
    std::lock_guard<std::mutex> g(s.mtx);
    s.events.push_back(e);
}

namespace {
/// stream-private blocks back to the shared cache (every queue drained first)
void flush_stream_free_locked(State& s) {
    if (s.stream_free.empty()) return;
    if (s.streams_ready)
        for (int i = 0; i < kNumQueues; ++i) slate_hip_call(hipStreamSynchronize(s.streams[i]));
    slate_hip_call(hipStreamSynchronize(nullptr));
    for (auto& kv : s.stream_free)
        for (auto& b : kv.second) { s.free_blocks.emplace(b.first, b.second); s.cached += b.first; }
    s.stream_free.clear();
    s.stream_cached = 0;
}

void* malloc_locked(State& s, size_t b) {
    if (!s.pending.empty()) reclaim_locked(s, false);
    auto it = s.free_blocks.find(b);
    void* p = nullptr;
    if (it != s.free_blocks.end()) {
        p = it->second;
        s.free_blocks.erase(it);
        s.cached -= b;
    } else {
        hipError_t e = hipMalloc(&p, b);
        if (e != hipSuccess) {
            // release every cache and retry once
            (void)hipGetLastError();
            reclaim_locked(s, true);
            flush_stream_free_locked(s);
            for (auto& kv : s.free_blocks) (void)hipFree(kv.second);
            ++g_free_epoch;
            s.free_blocks.clear();
            s.cached = 0;
            slate_hip_call(hipMalloc(&p, b));
        }
    }
    s.live[p] = b;
    s.in_use += b;
    return p;
}
}  // namespace

void* malloc(size_t bytes) {
    auto& s = st();
    void* p;
    {
        std::lock_guard<std::mutex> g(s.mtx);
        ensure_device_locked(s);
        p = malloc_locked(s, bucket(bytes));
    }
    own(p, &s);
    return p;
}

void* malloc_async(size_t bytes, hipStream_t stream) {
    auto& s = st();
    std::unique_lock<std::mutex> g(s.mtx);
    ensure_device_locked(s);
    const size_t b = bucket(bytes);
    void* p = nullptr;
    auto sf = s.stream_free.find(stream);
    if (sf != s.stream_free.end()) {
        auto it = sf->second.find(b);
        if (it != sf->second.end()) {
            p = it->second;
            sf->second.erase(it);
            s.stream_cached -= b;
            s.live[p] = b;
            s.in_use += b;
        }
    }
    if (!p) p = malloc_locked(s, b);
    s.live_stream[p] = stream;
    own(p, &s);
    return p;
}

namespace {
/// a block whose context was destroyed (its streams are gone): wait for the
/// context's device, hand the block back to HIP, and delete the context with
/// its last block.  Called with s.mtx held through `g`, which it releases.
void release_destroyed(State& s, void* ptr, std::unique_lock<std::mutex>& g) {
    int cur = -1;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(s.device);
    (void)hipDeviceSynchronize();
    (void)hipFree(ptr);
    ++g_free_epoch;
    if (cur >= 0) (void)hipSetDevice(cur);
    const bool last = s.live.empty();
    g.unlock();
    if (last) delete static_cast<Context*>(&s);
}
}  // namespace

void free_async(void* ptr, hipStream_t stream) {
    if (!ptr) return;
    auto& s = owner_of(ptr);
    std::unique_lock<std::mutex> g(s.mtx);
    auto it = s.live.find(ptr);
    slate_assert(it != s.live.end());
    const size_t b = it->second;
    s.live.erase(it);
    s.live_stream.erase(ptr);
    s.in_use -= b;
    if (s.destroyed) { release_destroyed(s, ptr, g); return; }
    s.stream_free[stream].emplace(b, ptr);
    s.stream_cached += b;
}

size_t bytes_stream_cached() { return st().stream_cached; }

void free(void* ptr) {
    if (!ptr) return;
    auto& s = owner_of(ptr);
    std::unique_lock<std::mutex> g(s.mtx);
    auto it = s.live.find(ptr);
    slate_assert(it != s.live.end());
    size_t b = it->second;
    s.live.erase(it);
    s.live_stream.erase(ptr);
    s.in_use -= b;
    if (s.destroyed) {
        // its context is gone (streams destroyed): release the block to HIP,
        // and the context itself with its last block
        release_destroyed(s, ptr, g);
        return;
    }
    if (!s.streams_ready) {
        // no queue ever ran: only synchronous (null-stream) use is possible
        slate_hip_call(hipStreamSynchronize(nullptr));
        s.free_blocks.emplace(b, ptr);
        s.cached += b;
        return;
    }
    // free on events: work already queued on any queue may still read the
    // block.  The null stream too -- except with CU-masked queues: those are
    // created blocking (hipExtStreamCreateWithCUMask takes no flags), so an
    // event on the legacy null stream would be a device-wide barrier between
    // the panel chain and the trailing update (profiles/r6_queue_overlap_probe.txt);
    // the library itself never works on the null stream.
    State::Pending pd{ptr, b, {}};
    const int nq = s.reserved_cus > 0 ? kNumQueues : kNumQueues + 1;
    pd.ev.reserve(nq);
    for (int i = 0; i < nq; ++i) {
        hipEvent_t e = event_get_locked(s);
        slate_hip_call(hipEventRecord(e, i < kNumQueues ? s.streams[i] : nullptr));
        pd.ev.push_back(e);
    }
    s.pending.push_back(std::move(pd));
}

void release_cache() {
    auto& s = st();
    std::lock_guard<std::mutex> g(s.mtx);
    reclaim_locked(s, true);
    flush_stream_free_locked(s);
    for (auto& kv : s.free_blocks) (void)hipFree(kv.second);
            ++g_free_epoch;
    s.free_blocks.clear();
    s.cached = 0;
}

size_t bytes_in_use() { return st().in_use; }
size_t bytes_cached() { return st().cached; }
size_t blocks_in_use() {
    auto& s = st();
    std::lock_guard<std::mutex> g(s.mtx);
    return s.live.size();
}
size_t blocks_cached() {
    auto& s = st();
    std::lock_guard<std::mutex> g(s.mtx);
    return s.free_blocks.size();
}
size_t host_bytes_in_use() { return st().host_in_use; }

void* malloc_host(size_t bytes) {
    void* p = nullptr;
    bytes = std::max<size_t>(bytes, 1);
    slate_hip_call(hipHostMalloc(&p, bytes, hipHostMallocDefault));
    auto& s = st();
    std::lock_guard<std::mutex> g(s.mtx);
    s.host_live[p] = bytes;
    s.host_in_use += bytes;
    return p;
}

void free_host(void* ptr) {
    if (!ptr) return;
    {
        auto& s = st();
        std::lock_guard<std::mutex> g(s.mtx);
        auto it = s.host_live.find(ptr);
        if (it != s.host_live.end()) {
            s.host_in_use -= it->second;
            s.host_live.erase(it);
        }
    }
    (void)hipHostFree(ptr);
}

void memcpy_async(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (bytes == 0) return;
    slate_hip_call(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s));
}

void memcpy2d_async(void* dst, size_t dpitch, const void* src, size_t spitch,
                    size_t width, size_t height, hipStream_t s) {
    if (width == 0 || height == 0) return;
    slate_hip_call(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDefault, s));
}

void memset_async(void* dst, int v, size_t bytes, hipStream_t s) {
    if (bytes == 0) return;
    slate_hip_call(hipMemsetAsync(dst, v, bytes, s));
}

}  // namespace device
}  // namespace slate
