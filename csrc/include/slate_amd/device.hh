// Device runtime: one GPU per rank (per process, or per in-process rank
// context), HIP streams/events, caching memory pool.
//
// Reference counterparts: BLAS++ Queue per device (MatrixStorage.hh:574-591:
// one comm queue + compute queues), Memory block pool (src/core/Memory.cc).
// Here: one process owns one MI355X; streams are created once per process and
// reused; device memory comes from a size-bucketed caching pool so drivers
// never call hipMalloc (which synchronises) in their hot loop.
#pragma once

#include "exception.hh"

#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>
#include <map>
#include <mutex>
#include <vector>

#define slate_hip_call(call) do {                                              \
    hipError_t _e = (call);                                                    \
    if (_e != hipSuccess)                                                      \
        throw ::slate::DeviceException(std::string(#call) + ": " +             \
              hipGetErrorString(_e), __func__, __FILE__, __LINE__);            \
    } while (0)

namespace slate {
namespace device {

/// Number of streams ("queues") per process: 0 = trailing update / default,
/// 1 = panel (high priority), 2 = lookahead columns, 3 = communication.
/// Exactly four, because HIP multiplexes streams onto GPU_MAX_HW_QUEUES
/// (4 by default) in-order hardware queues: more streams would alias onto
/// the same hardware queue and put panel kernels behind trailing GEMMs.
/// (The reference uses 2..3+lookahead BLAS++ queues, potrf.cc:66.)
constexpr int kNumQueues = 4;
constexpr int kCommQueue = 3;
constexpr int kLookaheadQueue = 2;
/// Trailing-update queue of the factorizations.
constexpr int kTrailQueue = 0;

/// True iff a HIP device is visible to this process.
bool available();
int  count();

/// Select the device used by this process (default: $LOCAL_RANK % count).
void set_device(int dev);
/// Did the program choose its device (set_device)?  Then the single-process
/// APIs stay on it instead of spreading over every visible GPU.
bool device_explicit();
int  get_device();

/// Device contexts (intra-process multi-GPU).  A context is one rank's view
/// of a device: its own stream set, event pool and allocator cache.  Every
/// thread uses the process context (device set_device / $LOCAL_RANK) unless
/// it has bound another one; in-process ranks (inproc.hh) bind one context
/// per rank thread, so N ranks on N GPUs -- or several ranks on one GPU --
/// each schedule onto their own queues.  Memory is returned to the context
/// that allocated it, whichever thread frees it.
struct Context;
/// New context on device `dev` (streams are created on first use).
Context* context_create(int dev);
/// Make `ctx` current for the calling thread (nullptr: the process context);
/// also makes its device current (hipSetDevice).
void context_bind(Context* ctx);
Context* context_current();
/// Synchronize the context's queues, release its cached memory and streams.
void context_destroy(Context* ctx);
int context_device(Context* ctx);

/// Stream set of the current context.  Queue 1 (panel) is created with high priority.
hipStream_t queue(int index);
void sync_all();
/// CUs reserved for the panel/comm queues (0 = no partitioning).
int reserved_cus();
/// A queue whose kernels may run on every CU: 0 without reservation, the
/// (unmasked) panel queue in shared mode.  Drivers without a panel chain
/// (SUMMA gemm) put their GEMMs there.
int full_queue();

/// Pooled event (disable-timing events for dependency edges).
hipEvent_t event_get();
void event_put(hipEvent_t e);

/// Caching device allocator.  Blocks are bucketed by rounded size and reused;
/// free is stream-ordered: the block is only handed out again once the work
/// queued before the free on every queue (and the null stream) has completed,
/// so early returns and exception paths cannot recycle memory under in-flight
/// kernels.
void* malloc(size_t bytes);
void  free(void* ptr);
/// Stream-ordered scratch: a block freed with free_async(p, s) is only
/// handed out again by malloc_async(.., s) on the same stream (stream order
/// makes immediate reuse safe), so per-call scratch of a kernel sequence on
/// one stream never reaches hipMalloc after the first call.  The block must
/// not be used by any other stream.
void* malloc_async(size_t bytes, hipStream_t s);
void  free_async(void* ptr, hipStream_t s);
size_t bytes_stream_cached();
void* malloc_host(size_t bytes);   // pinned host memory
void  free_host(void* ptr);
/// Number of times blocks went back to HIP (hipFree) so far: caches keyed by
/// device address (IPC handles) are stale once it changes.
uint64_t alloc_epoch();
/// Release all cached (unused) blocks back to HIP.
void  release_cache();
/// Bytes held in use / cached.
size_t bytes_in_use();
size_t bytes_cached();
/// Blocks handed out / parked in the cache; pinned host bytes handed out.
size_t blocks_in_use();
size_t blocks_cached();
size_t host_bytes_in_use();

void memcpy_async(void* dst, const void* src, size_t bytes, hipStream_t s);
void memcpy2d_async(void* dst, size_t dpitch, const void* src, size_t spitch,
                    size_t width, size_t height, hipStream_t s);
void memset_async(void* dst, int v, size_t bytes, hipStream_t s);

/// RAII typed device buffer from the pool.
template <typename T>
class Buffer {
public:
    Buffer() = default;
    explicit Buffer(size_t n) { resize(n); }
    // never throw out of a destructor (an exception already unwinding through
    // the owner would become std::terminate and hide the original error)
    ~Buffer() { try { reset(); } catch (...) {} }
    Buffer(Buffer const&) = delete;
    Buffer& operator=(Buffer const&) = delete;
    Buffer(Buffer&& o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
    Buffer& operator=(Buffer&& o) noexcept { reset(); p_ = o.p_; n_ = o.n_; o.p_ = nullptr; o.n_ = 0; return *this; }
    void resize(size_t n) {
        if (n <= n_) return;
        reset();
        p_ = static_cast<T*>(device::malloc(std::max<size_t>(n, 1) * sizeof(T)));
        n_ = n;
    }
    void reset() { if (p_) device::free(p_); p_ = nullptr; n_ = 0; }
    T* data() const { return p_; }
    size_t size() const { return n_; }
private:
    T* p_ = nullptr;
    size_t n_ = 0;
};

}  // namespace device
}  // namespace slate
