// Location-aware communication wrappers (staging) + SelfComm.
#include "slate_amd/comm.hh"

#include <cstring>
#include <map>

namespace slate {

namespace {

void local_copy(void* dst, const void* src, size_t bytes, Loc loc, hipStream_t s) {
    if (dst == src || bytes == 0) return;
    if (loc == Loc::Host) std::memcpy(dst, src, bytes);
    else device::memcpy_async(dst, src, bytes, s);
}

/// pinned host staging buffer, grown on demand (per thread)
struct HostStage {
    void* p = nullptr;
    size_t n = 0;
    void* get(size_t bytes) {
        if (bytes > n) {
            if (p) device::free_host(p);
            p = device::malloc_host(bytes);
            n = bytes;
        }
        return p;
    }
    ~HostStage() { /* leaked intentionally at exit */ }
};

void* host_stage(int slot, size_t bytes) {
    thread_local HostStage stages[4];
    return stages[slot].get(bytes);
}

}  // namespace

//------------------------------------------------------------------------------
void Comm::bcast(void* buf, size_t count, ScalarType t, int root, Loc loc, hipStream_t stream) {
    if (size() == 1 || count == 0) return;
    size_t bytes = count * scalar_size(t);
    if (device_native()) {
        if (loc == Loc::Device) { bcast_raw(buf, count, t, root, stream); return; }
        hipStream_t s = device::queue(device::kCommQueue);
        device::Buffer<char> tmp(bytes);
        device::memcpy_async(tmp.data(), buf, bytes, s);
        bcast_raw(tmp.data(), count, t, root, s);
        device::memcpy_async(buf, tmp.data(), bytes, s);
        slate_hip_call(hipStreamSynchronize(s));
        return;
    }
    if (loc == Loc::Host) { bcast_raw(buf, count, t, root, stream); return; }
    slate_hip_call(hipStreamSynchronize(stream));
    void* h = host_stage(0, bytes);
    if (rank() == root) {
        device::memcpy_async(h, buf, bytes, stream);
        slate_hip_call(hipStreamSynchronize(stream));
    }
    bcast_raw(h, count, t, root, nullptr);
    if (rank() != root) {
        device::memcpy_async(buf, h, bytes, stream);
        slate_hip_call(hipStreamSynchronize(stream));
    }
}

void Comm::allreduce(const void* send, void* recv, size_t count, ScalarType t, ReduceOp op,
                     Loc loc, hipStream_t stream) {
    if (count == 0) return;
    size_t bytes = count * scalar_size(t);
    if (size() == 1) { local_copy(recv, send, bytes, loc, stream); return; }
    if (device_native()) {
        if (loc == Loc::Device) { allreduce_raw(send, recv, count, t, op, stream); return; }
        hipStream_t s = device::queue(device::kCommQueue);
        device::Buffer<char> tmp(bytes);
        device::memcpy_async(tmp.data(), send, bytes, s);
        allreduce_raw(tmp.data(), tmp.data(), count, t, op, s);
        device::memcpy_async(recv, tmp.data(), bytes, s);
        slate_hip_call(hipStreamSynchronize(s));
        return;
    }
    if (loc == Loc::Host) { allreduce_raw(send, recv, count, t, op, stream); return; }
    slate_hip_call(hipStreamSynchronize(stream));
    void* h = host_stage(0, bytes);
    device::memcpy_async(h, send, bytes, stream);
    slate_hip_call(hipStreamSynchronize(stream));
    allreduce_raw(h, h, count, t, op, nullptr);
    device::memcpy_async(recv, h, bytes, stream);
    slate_hip_call(hipStreamSynchronize(stream));
}

void Comm::allgather(const void* send, void* recv, size_t count, ScalarType t, Loc loc, hipStream_t stream) {
    if (count == 0) return;
    size_t bytes = count * scalar_size(t);
    if (size() == 1) { local_copy(recv, send, bytes, loc, stream); return; }
    size_t total = bytes * size();
    if (device_native()) {
        if (loc == Loc::Device) { allgather_raw(send, recv, count, t, stream); return; }
        hipStream_t s = device::queue(device::kCommQueue);
        device::Buffer<char> tmp(bytes + total);
        device::memcpy_async(tmp.data(), send, bytes, s);
        allgather_raw(tmp.data(), tmp.data() + bytes, count, t, s);
        device::memcpy_async(recv, tmp.data() + bytes, total, s);
        slate_hip_call(hipStreamSynchronize(s));
        return;
    }
    if (loc == Loc::Host) { allgather_raw(send, recv, count, t, stream); return; }
    slate_hip_call(hipStreamSynchronize(stream));
    char* h = static_cast<char*>(host_stage(0, bytes + total));
    device::memcpy_async(h, send, bytes, stream);
    slate_hip_call(hipStreamSynchronize(stream));
    allgather_raw(h, h + bytes, count, t, nullptr);
    device::memcpy_async(recv, h + bytes, total, stream);
    slate_hip_call(hipStreamSynchronize(stream));
}

void Comm::exchange(std::vector<P2P> const& ops, ScalarType t, Loc loc, hipStream_t stream) {
    const size_t es = scalar_size(t);
    const int me = rank();
    // self pairs: i-th send to self matches i-th recv from self
    std::vector<const P2P*> self_send, self_recv, remote;
    for (auto const& o : ops) {
        if (o.peer == me) (o.is_send ? self_send : self_recv).push_back(&o);
        else remote.push_back(&o);
    }
    slate_assert(self_send.size() == self_recv.size());
    for (size_t i = 0; i < self_send.size(); ++i) {
        slate_assert(self_send[i]->count == self_recv[i]->count);
        local_copy(self_recv[i]->buf, self_send[i]->buf, self_send[i]->count * es, loc, stream);
    }
    if (remote.empty()) return;

    if (device_native() && loc == Loc::Device) {
        group_start();
        for (auto* o : remote) {
            if (o->is_send) send_raw(o->buf, o->count, t, o->peer, stream);
            else recv_raw(o->buf, o->count, t, o->peer, stream);
        }
        group_end();
        return;
    }
    if (!device_native() && loc == Loc::Host) {
        group_start();
        for (auto* o : remote) {
            if (o->is_send) send_raw(o->buf, o->count, t, o->peer, stream);
            else recv_raw(o->buf, o->count, t, o->peer, stream);
        }
        group_end();
        return;
    }
    // staging: copy every buffer to the transport's memory space
    size_t total = 0;
    for (auto* o : remote) total += o->count * es;
    if (device_native()) {
        hipStream_t s = device::queue(device::kCommQueue);
        device::Buffer<char> tmp(total);
        size_t off = 0;
        for (auto* o : remote) {
            if (o->is_send) device::memcpy_async(tmp.data() + off, o->buf, o->count * es, s);
            off += o->count * es;
        }
        group_start();
        off = 0;
        for (auto* o : remote) {
            if (o->is_send) send_raw(tmp.data() + off, o->count, t, o->peer, s);
            else recv_raw(tmp.data() + off, o->count, t, o->peer, s);
            off += o->count * es;
        }
        group_end();
        off = 0;
        for (auto* o : remote) {
            if (!o->is_send) device::memcpy_async(o->buf, tmp.data() + off, o->count * es, s);
            off += o->count * es;
        }
        slate_hip_call(hipStreamSynchronize(s));
        return;
    }
    slate_hip_call(hipStreamSynchronize(stream));
    char* h = static_cast<char*>(host_stage(1, total));
    size_t off = 0;
    for (auto* o : remote) {
        if (o->is_send) device::memcpy_async(h + off, o->buf, o->count * es, stream);
        off += o->count * es;
    }
    slate_hip_call(hipStreamSynchronize(stream));
    group_start();
    off = 0;
    for (auto* o : remote) {
        if (o->is_send) send_raw(h + off, o->count, t, o->peer, nullptr);
        else recv_raw(h + off, o->count, t, o->peer, nullptr);
        off += o->count * es;
    }
    group_end();
    off = 0;
    for (auto* o : remote) {
        if (!o->is_send) device::memcpy_async(o->buf, h + off, o->count * es, stream);
        off += o->count * es;
    }
    slate_hip_call(hipStreamSynchronize(stream));
}

//------------------------------------------------------------------------------
void SelfComm::allreduce_raw(const void*, void*, size_t, ScalarType, ReduceOp, hipStream_t) {}
void SelfComm::allgather_raw(const void*, void*, size_t, ScalarType, hipStream_t) {}
void SelfComm::send_raw(const void*, size_t, ScalarType, int, hipStream_t) {
    slate_error("SelfComm: send to another rank");
}
void SelfComm::recv_raw(void*, size_t, ScalarType, int, hipStream_t) {
    slate_error("SelfComm: recv from another rank");
}

}  // namespace slate
