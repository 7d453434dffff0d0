// RCCL transport: collectives and point-to-point over xGMI on device buffers,
// ordered on the caller's HIP stream.  Replaces the reference's MPI transport
// (hypercube listBcast in BaseMatrix.hh:2284-2386, MPI_Bcast/Allreduce sites).
#include "slate_amd/comm.hh"

#include <rccl/rccl.h>
#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <mutex>
#include <vector>

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
    /// All three are stream-ordered RCCL operations (kernels on the CUs).  The
    /// copy-engine path is the in-process transport (thread_comm.cc:
    /// hipMemcpyAsync peer copies).
    enum class BcastMode { Rccl, SendRecv, Tree };
    static BcastMode bcast_mode() {
        static const BcastMode m = [] {
            const char* e = std::getenv("SLATE_BCAST");
            std::string v = e ? e : "rccl";
            if (v == "sendrecv") return BcastMode::SendRecv;
            if (v == "tree") return BcastMode::Tree;
            slate_error_if_msg(v != "rccl", "SLATE_BCAST must be rccl, sendrecv or tree");
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
