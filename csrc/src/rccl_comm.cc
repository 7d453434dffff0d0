// RCCL transport: collectives and point-to-point over xGMI on device buffers,
// ordered on the caller's HIP stream.  Replaces the reference's MPI transport
// (hypercube listBcast in BaseMatrix.hh:2284-2386, MPI_Bcast/Allreduce sites).
#include "slate_amd/comm.hh"

#include <rccl/rccl.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#define slate_nccl_call(call) do {                                            \
    ncclResult_t _r = (call);                                                 \
    if (_r != ncclSuccess)                                                    \
        throw ::slate::CommException(std::string(#call) + ": " +              \
              ncclGetErrorString(_r), __func__, __FILE__, __LINE__);          \
    } while (0)

namespace slate {

namespace {

ncclDataType_t nccl_type(ScalarType t, size_t& mult) {
    mult = 1;
    switch (t) {
        case ScalarType::Int32:      return ncclInt32;
        case ScalarType::Int64:      return ncclInt64;
        case ScalarType::Float32:    return ncclFloat32;
        case ScalarType::Float64:    return ncclFloat64;
        case ScalarType::Complex64:  mult = 2; return ncclFloat32;
        case ScalarType::Complex128: mult = 2; return ncclFloat64;
        case ScalarType::Byte:       return ncclInt8;
    }
    return ncclInt8;
}

ncclRedOp_t nccl_op(ReduceOp op) {
    switch (op) {
        case ReduceOp::Sum: return ncclSum;
        case ReduceOp::Max: return ncclMax;
        case ReduceOp::Min: return ncclMin;
    }
    return ncclSum;
}

/// Every live communicator, so a watchdog can abort them all (comm_abort_all):
/// ncclCommAbort makes RCCL kernels stuck on a peer that never arrives return,
/// so a hung multi-GPU run ends with an error instead of holding its GPUs.
std::mutex g_reg_mtx;
std::vector<ncclComm_t>& registry() {
    static auto* v = new std::vector<ncclComm_t>();   // leaked: outlives static dtors
    return *v;
}
bool g_aborted = false;

//------------------------------------------------------------------------------
/// Copy-engine broadcast between the processes of one node (SLATE_BCAST=peer;
/// SURVEY §5.8, reference listBcast, include/slate/BaseMatrix.hh:2129-2212).
///
/// Every rank owns a ring of kStage staging buffers (hipMalloc'd and exported
/// once, re-exported only when a larger message outgrows one) and maps every
/// other rank's buffers once.  Every rank sees every broadcast of the
/// communicator in the same order (collective semantics), so each one knows,
/// without asking, the root's message number rm and with it the staging slot
/// rm % kStage and event slot rm % kRing.  One broadcast:
///   root:     (slot reuse) waits until every receiver has issued its copy out
///             of the slot's previous message and (wait_ipc) on each
///             receiver's latest copy; copies the message into the
///             staging slot on its stream, records ready[rm % kRing],
///             publishes (seq, bytes) -- and returns: its buffer is free;
///   receiver: waits (host) for the root's seq, then on its single copy
///             stream: after the root's ready event (wait_ipc) and the
///             caller's stream (buffer reuse), PULLS the bytes with one hipMemcpyAsync
///             from the mapped staging buffer -- an SDMA copy over xGMI, no
///             kernel on the CUs the trailing GEMM is using -- records its
///             interprocess done event (for the root) and a plain event the
///             caller's stream waits on.  Waits on interprocess events go
///             through wait_ipc (query, stream wait, host poll as the last
///             resort).
/// One copy stream per receiver makes "latest done event complete" imply
/// every earlier copy complete, which is what the root's slot reuse needs.
/// The host of the root waits only when the receivers lag kStage of its
/// messages behind.  No handle depends on the lifetime of the caller's
/// buffers.  The control block is a POSIX shared-memory segment named by
/// rank 0 (one ncclBroadcast at set-up); a communicator whose ranks cannot
/// map each other's memory / events keeps ncclBroadcast (the ranks agree
/// through an all-reduce).
class PeerBcast {
public:
    static constexpr int kMaxRanks = 64, kRing = 16, kStage = 4;
    struct Stage { hipIpcMemHandle_t mem; uint64_t id, cap; };
    struct Msg { std::atomic<uint64_t> seq; uint64_t bytes; };
    struct alignas(64) Slot {
        std::atomic<uint64_t> done_seq;    // every broadcast up to this one processed
        std::atomic<int> last_done;        // event slot of my latest receive copy (-1: none)
        std::atomic<int> inited;
        Msg msg[kStage];                   // my messages as root, by staging slot
        Stage st[kStage];                  // my staging buffers
        hipIpcEventHandle_t ready_ev[kRing], done_ev[kRing];
    };
    struct Block { Slot r[kMaxRanks]; };

    /// Collective set-up over `comm`; ok() is false on every rank when any
    /// rank could not map the control block, export / import interprocess
    /// events or open a peer's staging memory.
    PeerBcast(ncclComm_t comm, int rank, int size) : rank_(rank), size_(size), count_(size, 0) {
        hipStream_t st = device::queue(device::kCommQueue);
        auto allmin = [&](int v) {
            device::Buffer<int> d(1);
            device::memcpy_async(d.data(), &v, sizeof v, st);
            slate_nccl_call(ncclAllReduce(d.data(), d.data(), 1, ncclInt32, ncclMin, comm, st));
            device::memcpy_async(&v, d.data(), sizeof v, st);
            slate_hip_call(hipStreamSynchronize(st));
            return v;
        };
        // rank 0 names and creates the segment, the others learn the name
        char name[64] = {};
        if (rank == 0) {
            static std::atomic<int> counter{0};
            std::snprintf(name, sizeof name, "/slate_pb_%d_%d", int(getpid()), counter++);
            int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
            if (fd < 0 || ftruncate(fd, sizeof(Block)) != 0) name[0] = 0;
            if (fd >= 0) close(fd);
        }
        {
            device::Buffer<char> d(sizeof name);
            device::memcpy_async(d.data(), name, sizeof name, st);
            slate_nccl_call(ncclBroadcast(d.data(), d.data(), sizeof name, ncclInt8, 0, comm, st));
            device::memcpy_async(name, d.data(), sizeof name, st);
            slate_hip_call(hipStreamSynchronize(st));
        }
        int ok = size <= kMaxRanks && name[0] != 0;
        if (ok) {
            int fd = shm_open(name, O_RDWR, 0600);
            void* p = fd >= 0 ? mmap(nullptr, sizeof(Block), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0) : MAP_FAILED;
            if (fd >= 0) close(fd);
            if (p == MAP_FAILED) ok = 0;
            else blk_ = static_cast<Block*>(p);
        }
        if (ok) {
            try {
                Slot& me = blk_->r[rank_];
                me.last_done.store(-1, std::memory_order_relaxed);
                for (int i = 0; i < kRing; ++i) {
                    slate_hip_call(hipEventCreateWithFlags(&ready_[i], hipEventDisableTiming | hipEventInterprocess));
                    slate_hip_call(hipEventCreateWithFlags(&done_[i], hipEventDisableTiming | hipEventInterprocess));
                    slate_hip_call(hipIpcGetEventHandle(&me.ready_ev[i], ready_[i]));
                    slate_hip_call(hipIpcGetEventHandle(&me.done_ev[i], done_[i]));
                    slate_hip_call(hipEventCreateWithFlags(&fork_[i], hipEventDisableTiming));
                    slate_hip_call(hipEventCreateWithFlags(&local_[i], hipEventDisableTiming));
                }
                slate_hip_call(hipStreamCreateWithFlags(&cs_, hipStreamNonBlocking));
                for (int j = 0; j < kStage; ++j) grow(j, size_t(1) << 20);   // 1 MiB to start
                me.inited.store(1, std::memory_order_release);
            } catch (std::exception const&) { ok = 0; }
        }
        ok = allmin(ok);
        if (ok) {
            try {   // every rank maps every other rank's events and staging buffers once
                for (int r = 0; r < size_; ++r) {
                    spin([&] { return blk_->r[r].inited.load(std::memory_order_acquire) != 0; });
                    if (r == rank_) continue;
                    (void)imported(r, 0, true);
                    (void)imported(r, 0, false);
                    for (int j = 0; j < kStage; ++j) (void)staged(r, j);
                }
            } catch (std::exception const&) { ok = 0; }
            ok = allmin(ok);   // also: every rank mapped the segment, the name can go
        }
        if (rank == 0 && name[0]) shm_unlink(name);
        ok_ = ok != 0;
        if (ok_ && rank == 0 && std::getenv("SLATE_BCAST_VERBOSE"))
            std::fprintf(stderr, "slate: SLATE_BCAST=peer active on a communicator of %d ranks\n", size);
        if (!ok_ && rank == 0) {
            static std::once_flag warned;
            std::call_once(warned, [] {
                std::fprintf(stderr, "slate: SLATE_BCAST=peer unavailable (interprocess memory / events); "
                                     "using ncclBroadcast\n");
            });
        }
    }
    bool ok() const { return ok_; }
    ~PeerBcast() {
        // at interpreter exit the HIP runtime may be gone: unmap the control
        // block only (staging memory goes with the process)
        if (blk_) munmap(blk_, sizeof(Block));
    }

    void bcast(void* buf, size_t bytes, int root, hipStream_t s) {
        const uint64_t seq = ++seq_;
        const uint64_t rm = count_[root]++;                   // the root's message number
        const int j = int(rm % kStage), e = int(rm % kRing);
        Block& B = *blk_;
        Slot& me = B.r[rank_];
        if (rank_ == root) {
            if (rm >= uint64_t(kStage)) {
                // staging slot j carried message stage_seq_[j]: every receiver
                // has issued its copy out of it (host), and its copy stream
                // finished it (GPU: its latest done event)
                const uint64_t prev = stage_seq_[j];
                for (int r = 0; r < size_; ++r) {
                    if (r == rank_) continue;
                    spin([&] { return B.r[r].done_seq.load(std::memory_order_acquire) >= prev; });
                    const int ld = B.r[r].last_done.load(std::memory_order_acquire);
                    if (ld < 0) continue;
                    // kStage messages later that copy has almost always finished
                    wait_ipc(s, imported(r, ld, false));
                }
            }
            if (bytes > stage_cap_[j]) grow(j, bytes);
            slate_hip_call(hipMemcpyAsync(stage_[j], buf, bytes, hipMemcpyDeviceToDevice, s));
            slate_hip_call(hipEventRecord(ready_[e], s));
            me.msg[j].bytes = bytes;
            me.msg[j].seq.store(seq, std::memory_order_release);
            stage_seq_[j] = seq;
            me.done_seq.store(seq, std::memory_order_release);
            return;
        }
        Msg& msg = B.r[root].msg[j];
        spin([&] { return msg.seq.load(std::memory_order_acquire) == seq; });
        slate_error_if_msg(msg.bytes != bytes, "SLATE_BCAST=peer: broadcast sizes differ between ranks");
        char* src = static_cast<char*>(staged(root, j));
        const int f = int(recv_ % kRing);
        ++recv_;
        slate_hip_call(hipEventRecord(fork_[f], s));              // buf's earlier users on the caller's stream
        slate_hip_call(hipStreamWaitEvent(cs_, fork_[f], 0));
        wait_ipc(cs_, imported(root, e, true));                    // the root's staging copy
        slate_hip_call(hipMemcpyAsync(buf, src, bytes, hipMemcpyDeviceToDevice, cs_));
        slate_hip_call(hipEventRecord(done_[f], cs_));         // for the root (interprocess)
        slate_hip_call(hipEventRecord(local_[f], cs_));        // for this process's stream
        slate_hip_call(hipStreamWaitEvent(s, local_[f], 0));
        me.last_done.store(f, std::memory_order_release);
        me.done_seq.store(seq, std::memory_order_release);
    }

private:
    template <typename F>
    void spin(F&& ready) {
        // a peer that never arrives is a hung job: fail loudly instead of spinning forever
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; !ready(); ++i) {
            if (i > 64) std::this_thread::yield();
            if ((i & 1023) == 1023 &&
                std::chrono::steady_clock::now() - t0 > std::chrono::seconds(600))
                throw CommException("SLATE_BCAST=peer: a peer did not arrive within 600 s", __func__, __FILE__,
                                    __LINE__);
        }
    }
    /// Make stream `s` wait for an interprocess event.  A completed event
    /// needs nothing.  A stream wait on an imported event that is still
    /// pending failed on the shared-GPU rig with "invalid argument"
    /// (profiles/r6_bench_verify.txt); then the host polls it instead -- on
    /// this rank's comm lane only, and only in that case, since a host that
    /// blocks on GPU progress can deadlock against collectives that other
    /// ranks have not issued yet.
    void wait_ipc(hipStream_t s, hipEvent_t ev) {
        hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) slate_hip_call(q);
        if (hipStreamWaitEvent(s, ev, 0) == hipSuccess) return;
        (void)hipGetLastError();
        spin([&] {
            q = hipEventQuery(ev);
            if (q == hipSuccess) return true;
            if (q != hipErrorNotReady) slate_hip_call(q);
            return false;
        });
    }
    /// (re)allocate and export my staging buffer j; an outgrown buffer stays
    /// allocated (receivers may still read it; sizes only grow, so this
    /// happens a few times per communicator)
    void grow(int j, size_t bytes) {
        const size_t cap = std::max<size_t>(bytes, stage_cap_[j] * 2);
        void* p = nullptr;
        slate_hip_call(hipMalloc(&p, cap));
        stage_[j] = static_cast<char*>(p);
        stage_cap_[j] = cap;
        Stage& st = blk_->r[rank_].st[j];
        slate_hip_call(hipIpcGetMemHandle(&st.mem, p));
        st.cap = cap;
        st.id = ++stage_ids_;
    }
    /// rank r's staging buffer j mapped here (re-mapped when r grew it; the
    /// old mapping stays: copies from it may still be queued)
    void* staged(int r, int j) {
        Stage const& st = blk_->r[r].st[j];
        auto& m = mapped_[r * kStage + j];
        if (!m.first || m.second != st.id) {
            void* p = nullptr;
            slate_hip_call(hipIpcOpenMemHandle(&p, st.mem, hipIpcMemLazyEnablePeerAccess));
            m = {p, st.id};
        }
        return m.first;
    }
    hipEvent_t imported(int r, int slot, bool ready) {
        auto& m = ready ? imp_ready_ : imp_done_;
        const int key = r * kRing + slot;
        auto it = m.find(key);
        if (it != m.end()) return it->second;
        hipEvent_t e;
        slate_hip_call(hipIpcOpenEventHandle(&e, ready ? blk_->r[r].ready_ev[slot] : blk_->r[r].done_ev[slot]));
        m[key] = e;
        return e;
    }

    int rank_, size_;
    bool ok_ = false;
    Block* blk_ = nullptr;
    uint64_t seq_ = 0, recv_ = 0, stage_ids_ = 0;
    std::vector<uint64_t> count_;                 // messages rooted at each rank so far
    uint64_t stage_seq_[kStage] = {};
    hipEvent_t ready_[kRing] = {}, done_[kRing] = {}, fork_[kRing] = {}, local_[kRing] = {};
    hipStream_t cs_ = nullptr;                    // my single copy stream (receiver)
    char* stage_[kStage] = {};
    size_t stage_cap_[kStage] = {};
    std::map<int, std::pair<void*, uint64_t>> mapped_;
    std::map<int, hipEvent_t> imp_ready_, imp_done_;
};

class RcclComm : public Comm {
public:
    RcclComm(ncclComm_t c) : comm_(c) {
        slate_nccl_call(ncclCommCount(comm_, &size_));
        slate_nccl_call(ncclCommUserRank(comm_, &rank_));
        std::lock_guard<std::mutex> l(g_reg_mtx);
        registry().push_back(comm_);
    }
    ~RcclComm() override {
        bool aborted;
        {
            std::lock_guard<std::mutex> l(g_reg_mtx);
            auto& r = registry();
            r.erase(std::remove(r.begin(), r.end(), comm_), r.end());
            aborted = g_aborted;
        }
        // Destroy only if the process is still healthy; at interpreter exit the
        // HIP runtime may already be torn down.  An aborted comm is gone.
        if (comm_ && !aborted) (void)ncclCommDestroy(comm_);
    }
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    std::string name() const override { return "rccl"; }
    bool device_native() const override { return true; }
    int device() const override {
        int d = -1;
        return ncclCommCuDevice(comm_, &d) == ncclSuccess ? d : -1;
    }
    ncclComm_t raw() const { return comm_; }

    /// Broadcast transport (SLATE_BCAST, read once; reference: listBcast's
    /// radix-2 / radix-4 hypercube trees over point-to-point messages,
    /// include/slate/BaseMatrix.hh:2129-2212, 2326-2386):
    ///   rccl     ncclBroadcast (RCCL's pipelined ring / tree; default)
    ///   sendrecv flat fan-out: the root sends to every peer in ONE group --
    ///            on the fully connected xGMI mesh each message has its own link
    ///   tree     binomial tree of grouped send / recv, log2(n) rounds
    ///   peer     copy-engine pull of the root's buffer (PeerBcast above):
    ///            no kernel on the CUs; processes of one node
    /// The first three are stream-ordered RCCL operations (kernels on the CUs).
    enum class BcastMode { Rccl, SendRecv, Tree, Peer };
    /// Default: peer (the panel broadcasts then take no CUs from the trailing
    /// GEMM: profiles/r6_critpath_2x4_cus_nonblocking.txt, CU-free messages);
    /// a communicator whose ranks cannot map each other's memory keeps
    /// ncclBroadcast by itself (PeerBcast::ok).
    static BcastMode bcast_mode() {
        static const BcastMode m = [] {
            const char* e = std::getenv("SLATE_BCAST");
            std::string v = e ? e : "peer";
            if (v == "sendrecv") return BcastMode::SendRecv;
            if (v == "tree") return BcastMode::Tree;
            if (v == "peer") return BcastMode::Peer;
            slate_error_if_msg(v != "rccl", "SLATE_BCAST must be rccl, sendrecv, tree or peer");
            return BcastMode::Rccl;
        }();
        return m;
    }

    void bcast_raw(void* buf, size_t count, ScalarType t, int root, hipStream_t s) override {
        size_t mult;
        auto dt = nccl_type(t, mult);
        const size_t n = count * mult;
        if (size_ == 1 || n == 0) return;
        switch (bcast_mode()) {
            case BcastMode::Peer:
                if (!peer_) peer_ = std::make_unique<PeerBcast>(comm_, rank_, size_);
                if (peer_->ok()) {
                    peer_->bcast(buf, count * scalar_size(t), root, s);
                    return;
                }
                slate_nccl_call(ncclBroadcast(buf, buf, n, dt, root, comm_, s));
                return;
            case BcastMode::Rccl:
                slate_nccl_call(ncclBroadcast(buf, buf, n, dt, root, comm_, s));
                return;
            case BcastMode::SendRecv:
                slate_nccl_call(ncclGroupStart());
                if (rank_ == root) {
                    for (int d = 1; d < size_; ++d)
                        slate_nccl_call(ncclSend(buf, n, dt, (root + d) % size_, comm_, s));
                } else {
                    slate_nccl_call(ncclRecv(buf, n, dt, root, comm_, s));
                }
                slate_nccl_call(ncclGroupEnd());
                return;
            case BcastMode::Tree: {
                const int vr = (rank_ - root + size_) % size_;   // rank relative to the root
                for (int mask = 1; mask < size_; mask <<= 1) {
                    if (vr < mask && vr + mask < size_) {
                        slate_nccl_call(ncclSend(buf, n, dt, (vr + mask + root) % size_, comm_, s));
                    } else if (vr >= mask && vr < 2 * mask) {
                        slate_nccl_call(ncclRecv(buf, n, dt, (vr - mask + root) % size_, comm_, s));
                    }
                }
                return;
            }
        }
    }
    void allreduce_raw(const void* send, void* recv, size_t count, ScalarType t,
                       ReduceOp op, hipStream_t s) override {
        size_t mult;
        auto dt = nccl_type(t, mult);
        slate_error_if_msg(mult != 1 && op != ReduceOp::Sum, "complex max/min allreduce");
        slate_nccl_call(ncclAllReduce(send, recv, count * mult, dt, nccl_op(op), comm_, s));
    }
    void allgather_raw(const void* send, void* recv, size_t count, ScalarType t, hipStream_t s) override {
        size_t mult;
        auto dt = nccl_type(t, mult);
        slate_nccl_call(ncclAllGather(send, recv, count * mult, dt, comm_, s));
    }
    void send_raw(const void* buf, size_t count, ScalarType t, int peer, hipStream_t s) override {
        size_t mult;
        auto dt = nccl_type(t, mult);
        slate_nccl_call(ncclSend(buf, count * mult, dt, peer, comm_, s));
    }
    void recv_raw(void* buf, size_t count, ScalarType t, int peer, hipStream_t s) override {
        size_t mult;
        auto dt = nccl_type(t, mult);
        slate_nccl_call(ncclRecv(buf, count * mult, dt, peer, comm_, s));
    }
    void group_start() override { slate_nccl_call(ncclGroupStart()); }
    void group_end() override { slate_nccl_call(ncclGroupEnd()); }
    void barrier() override {
        // a 1-element allreduce on the comm stream, then wait for it
        hipStream_t s = device::queue(device::kCommQueue);
        device::Buffer<int> one(1);
        device::memset_async(one.data(), 0, sizeof(int), s);
        slate_nccl_call(ncclAllReduce(one.data(), one.data(), 1, ncclInt32, ncclSum, comm_, s));
        slate_hip_call(hipStreamSynchronize(s));
    }

private:
    ncclComm_t comm_ = nullptr;
    int rank_ = 0, size_ = 1;
    std::unique_ptr<PeerBcast> peer_;
};

}  // namespace

int comm_abort_all() {
    std::vector<ncclComm_t> v;
    {
        std::lock_guard<std::mutex> l(g_reg_mtx);
        v = registry();
        g_aborted = true;
    }
    for (ncclComm_t c : v) (void)ncclCommAbort(c);
    return int(v.size());
}

std::string comm_async_errors() {
    std::vector<ncclComm_t> v;
    {
        std::lock_guard<std::mutex> l(g_reg_mtx);
        v = registry();
    }
    std::string out;
    for (ncclComm_t c : v) {
        ncclResult_t r = ncclSuccess;
        if (ncclCommGetAsyncError(c, &r) == ncclSuccess && r != ncclSuccess && r != ncclInProgress) {
            if (!out.empty()) out += "; ";
            out += ncclGetErrorString(r);
        }
    }
    return out;
}

std::string rccl_unique_id() {
    ncclUniqueId id;
    slate_nccl_call(ncclGetUniqueId(&id));
    return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

CommPtr make_rccl_comm(std::string const& unique_id, int nranks, int rank) {
    slate_error_if_msg(unique_id.size() != NCCL_UNIQUE_ID_BYTES, "bad RCCL unique id size");
    ncclUniqueId id;
    std::memcpy(id.internal, unique_id.data(), NCCL_UNIQUE_ID_BYTES);
    device::get_device();  // bind this process's GPU before init
    ncclComm_t c;
    slate_nccl_call(ncclCommInitRank(&c, nranks, id, rank));
    return std::make_shared<RcclComm>(c);
}

CommPtr rccl_split(CommPtr const& parent, int color, int key) {
    auto* p = dynamic_cast<RcclComm*>(parent.get());
    slate_error_if_msg(!p, "rccl_split: parent is not an RCCL communicator");
    ncclComm_t c = nullptr;
    slate_nccl_call(ncclCommSplit(p->raw(), color, key, &c, nullptr));
    if (!c) return nullptr;
    return std::make_shared<RcclComm>(c);
}

}  // namespace slate
