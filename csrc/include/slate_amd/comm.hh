// Communication layer.
//
// Reference: MPI everywhere (BaseMatrix.hh listBcast/listReduce hypercubes,
// internal_comm.cc, MPI_Bcast/Allreduce call sites listed in SURVEY §2.3.1).
// Here: one process per GPU; an abstract Comm with three transports:
//   * RcclComm  - RCCL over xGMI, device buffers, stream-ordered (production).
//   * HostComm  - a host transport supplied by the embedding runtime (the
//                 Python layer plugs torch.distributed/gloo in through the
//                 bindings).  Device buffers are staged through pinned host
//                 memory, like the reference's non-GPU-aware-MPI path.
//   * SelfComm  - single rank (the reference's mpi_stubs.cc analog).
// Every rank must issue collectives on a communicator in the same order;
// drivers issue all communication in program order on one comm stream.
#pragma once

#include "types.hh"
#include "device.hh"

#include <memory>
#include <string>
#include <vector>

namespace slate {

enum class ReduceOp : char { Sum = 's', Max = 'x', Min = 'n' };

inline size_t scalar_size(ScalarType t) {
    switch (t) {
        case ScalarType::Int32: return 4;
        case ScalarType::Int64: return 8;
        case ScalarType::Float32: return 4;
        case ScalarType::Float64: return 8;
        case ScalarType::Complex64: return 8;
        case ScalarType::Complex128: return 16;
        case ScalarType::Byte: return 1;
    }
    return 1;
}

/// Where a buffer handed to a Comm lives.
enum class Loc : char { Host = 'H', Device = 'D' };

class Comm {
public:
    virtual ~Comm() = default;
    virtual int rank() const = 0;
    virtual int size() const = 0;
    virtual std::string name() const = 0;

    /// Can the transport read/write device memory directly (stream-ordered)?
    virtual bool device_native() const { return false; }
    /// HIP device the communicator is bound to (RCCL: ncclCommCuDevice), -1 if none.
    virtual int device() const { return -1; }

    // ---- raw transport operations (buffers in the transport's native space:
    // device memory if device_native(), else host memory).  `stream` orders
    // device-native operations; host transports are synchronous.
    virtual void bcast_raw(void* buf, size_t count, ScalarType t, int root, hipStream_t stream) = 0;
    virtual void allreduce_raw(const void* send, void* recv, size_t count, ScalarType t,
                               ReduceOp op, hipStream_t stream) = 0;
    virtual void allgather_raw(const void* send, void* recv, size_t count, ScalarType t,
                               hipStream_t stream) = 0;
    virtual void send_raw(const void* buf, size_t count, ScalarType t, int peer, hipStream_t stream) = 0;
    virtual void recv_raw(void* buf, size_t count, ScalarType t, int peer, hipStream_t stream) = 0;
    /// Group several send/recv so they progress concurrently (ncclGroupStart/End).
    virtual void group_start() {}
    virtual void group_end() {}
    virtual void barrier() = 0;

    // ---- location-aware wrappers: stage through host or device as needed.
    void bcast(void* buf, size_t count, ScalarType t, int root, Loc loc, hipStream_t stream);
    void allreduce(const void* send, void* recv, size_t count, ScalarType t, ReduceOp op,
                   Loc loc, hipStream_t stream);
    void allgather(const void* send, void* recv, size_t count, ScalarType t, Loc loc, hipStream_t stream);

    /// Exchange: a batch of sends and receives that progress together.
    struct P2P { void* buf; size_t count; int peer; bool is_send; };
    void exchange(std::vector<P2P> const& ops, ScalarType t, Loc loc, hipStream_t stream);

    template <typename T>
    void bcast(T* buf, size_t count, int root, Loc loc, hipStream_t s) {
        bcast(static_cast<void*>(buf), count, scalar_type<T>(), root, loc, s);
    }
    template <typename T>
    void allreduce(T* buf, size_t count, ReduceOp op, Loc loc, hipStream_t s) {
        allreduce(buf, buf, count, scalar_type<T>(), op, loc, s);
    }
    /// Host scalar convenience.
    template <typename T>
    T allreduce_scalar(T v, ReduceOp op) {
        allreduce(&v, &v, 1, scalar_type<T>(), op, Loc::Host, nullptr);
        return v;
    }
};

using CommPtr = std::shared_ptr<Comm>;

/// Single-rank communicator.
class SelfComm : public Comm {
public:
    int rank() const override { return 0; }
    int size() const override { return 1; }
    std::string name() const override { return "self"; }
    bool device_native() const override { return true; }  // no-ops work on any memory
    void bcast_raw(void*, size_t, ScalarType, int, hipStream_t) override {}
    void allreduce_raw(const void* s, void* r, size_t c, ScalarType t, ReduceOp, hipStream_t st) override;
    void allgather_raw(const void* s, void* r, size_t c, ScalarType t, hipStream_t st) override;
    void send_raw(const void*, size_t, ScalarType, int, hipStream_t) override;
    void recv_raw(void*, size_t, ScalarType, int, hipStream_t) override;
    void barrier() override {}
};

/// Host transport implemented by a callback object (Python torch.distributed
/// bindings, or a test harness).  All buffers passed to the *_raw methods are
/// host pointers.
class HostComm : public Comm {
public:
    std::string name() const override { return "host"; }
    bool device_native() const override { return false; }
};

/// Create an RCCL communicator from a 128-byte unique id (exchanged by the
/// embedding runtime) for `nranks` ranks.  Throws if RCCL is unavailable.
CommPtr make_rccl_comm(std::string const& unique_id, int nranks, int rank);
/// Create an RCCL unique id (call on one rank, distribute the bytes).
std::string rccl_unique_id();
/// Split an RCCL communicator (ncclCommSplit); collective over `parent`.
CommPtr rccl_split(CommPtr const& parent, int color, int key);
/// In-process communicators (thread_comm.cc): `n` ranks that are threads of
/// one process; element r is rank r's endpoint, to be used by one thread.
/// device_mode: buffers are device memory of the ranks' contexts and data
/// moves by peer copies ordered with events; else host memory (memcpy).
std::vector<CommPtr> make_thread_comms(int n, bool device_mode);
/// Wake every rank blocked on this in-process communicator with an exception
/// (a rank failed); no-op for other transports.
void thread_comm_abort(Comm& c);

/// Abort every live RCCL communicator of this process (ncclCommAbort; safe
/// from a watchdog thread while another thread waits on a stuck collective).
/// Returns how many were aborted; the communicators are unusable afterwards.
int comm_abort_all();
/// Asynchronous errors reported by the live RCCL communicators ("" if none).
std::string comm_async_errors();

}  // namespace slate
