// In-process communicator: the ranks of a grid are threads of ONE process,
// each driving its own device context (device.hh), so a single-process
// program -- the LAPACK-compatible API, a C++ or Python script -- uses every
// GPU of the node.  The reference reaches the same end by spreading one MPI
// rank's tiles over all of its GPUs (tileDevice = device_1d_grid,
// include/slate/internal/MatrixStorage.hh:503-511) with host-thread
// parallelism inside every internal op; here each GPU is a rank of the
// ordinary p x q machinery and only the transport differs.
//
// Transport (device mode): a host rendezvous per operation publishes buffer
// pointers and HIP events; data then moves by peer copies (hipMemcpyAsync
// between devices: the SDMA engines over xGMI, no CUs taken from the
// trailing GEMM -- SURVEY §5.8's CU-free broadcast), ordered on the callers'
// streams by cross-device hipStreamWaitEvent.  Every event is recorded
// before any rank waits on it and no GPU wait depends on a later host
// action, so the GPU side cannot deadlock; the host side has the ordering
// rules of a blocking host transport (every communicator sees its
// operations in one program order).  Reductions copy the ranks' buffers into
// staging slabs and reduce them with one kernel (kernels/comm.hip).  Host
// mode (no GPU, CPU builds and tests): the same rendezvous with memcpy.
#include "slate_amd/comm.hh"
#include "slate_amd/grid.hh"
#include "../kernels/kernels.hh"

#include <algorithm>
#include <complex>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <string>
#include <deque>
#include <map>
#include <mutex>

namespace slate {

namespace {

hipEvent_t record(hipStream_t s) {
    hipEvent_t e;
    slate_hip_call(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    slate_hip_call(hipEventRecord(e, s));
    return e;
}
void wait_on(hipStream_t s, hipEvent_t e) { if (e) slate_hip_call(hipStreamWaitEvent(s, e, 0)); }
void destroy(hipEvent_t& e) { if (e) (void)hipEventDestroy(e); e = nullptr; }

struct Hub {
    int n;
    bool dev;
    std::mutex m;
    std::condition_variable cv;
    uint64_t gen = 0;
    int arrived = 0;
    bool aborted = false;
    struct Slot { const void* ptr = nullptr; hipEvent_t ev = nullptr; };
    // phase A: data ready; phase B: reads done; phase C: the sliced
    // all-reduce's last hand-off.  C is written by no collective before its
    // first barrier, so a fast rank that has already entered the next
    // collective (and rewritten its A slot) cannot clobber the event a slow
    // rank still has to read after barrier (3) of allreduce_sliced.
    std::vector<Slot> a, b, c;
    struct Msg {
        const void* ptr;
        size_t bytes;
        hipEvent_t ev;
        hipEvent_t done = nullptr;
        bool completed = false;
    };
    std::map<std::pair<int, int>, std::deque<std::shared_ptr<Msg>>> box;   // (src, dst) FIFO

    Hub(int n_, bool d) : n(n_), dev(d), a(n_), b(n_), c(n_) {}

    void check() {
        if (aborted) throw CommException("in-process communicator aborted (another rank failed)", __func__,
                                         __FILE__, __LINE__);
    }
    void barrier() {
        std::unique_lock<std::mutex> l(m);
        check();
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return;
        }
        cv.wait(l, [&] { return gen != g || aborted; });
        check();
    }
    void abort() {
        std::lock_guard<std::mutex> l(m);
        aborted = true;
        cv.notify_all();
    }
    /// back to a clean state after an aborted run (every rank thread joined):
    /// persistent in-process groups reuse their communicators
    void reset() {
        std::lock_guard<std::mutex> l(m);
        aborted = false;
        arrived = 0;
        box.clear();
    }
};

char type_char(ScalarType t, size_t& mult) {
    mult = 1;
    switch (t) {
        case ScalarType::Float32: return 'f';
        case ScalarType::Float64: return 'd';
        case ScalarType::Int32: return 'i';
        case ScalarType::Int64: return 'l';
        case ScalarType::Byte: return 'b';
        case ScalarType::Complex64: mult = 2; return 'f';
        case ScalarType::Complex128: mult = 2; return 'd';
    }
    return 'b';
}

template <typename T>
void host_reduce(T* out, std::vector<const void*> const& in, size_t count, ReduceOp op) {
    for (size_t i = 0; i < count; ++i) {
        T acc = static_cast<const T*>(in[0])[i];
        for (size_t r = 1; r < in.size(); ++r) {
            const T x = static_cast<const T*>(in[r])[i];
            if (op == ReduceOp::Sum) acc += x;
            else if (op == ReduceOp::Max) acc = x > acc ? x : acc;
            else acc = x < acc ? x : acc;
        }
        out[i] = acc;
    }
}

class ThreadComm : public Comm {
public:
    ThreadComm(std::shared_ptr<Hub> hub, int rank) : hub_(std::move(hub)), me_(rank) {}
    ~ThreadComm() override { destroy(pend_b_); }
    int rank() const override { return me_; }
    int size() const override { return hub_->n; }
    std::string name() const override { return "inproc"; }
    bool device_native() const override { return hub_->dev; }
    void abort() { hub_->abort(); }
    void reset() { hub_->reset(); }

    void bcast_raw(void* buf, size_t count, ScalarType t, int root, hipStream_t s) override {
        const size_t bytes = count * scalar_size(t);
        Hub& h = *hub_;
        if (!h.dev) {
            h.a[me_].ptr = buf;
            h.barrier();
            if (me_ != root) std::memcpy(buf, h.a[root].ptr, bytes);
            h.barrier();
            return;
        }
        h.a[me_] = {buf, me_ == root ? record(s) : nullptr};
        h.barrier();
        destroy(pend_b_);
        hipEvent_t mine = nullptr;
        if (me_ != root) {
            wait_on(s, h.a[root].ev);
            device::memcpy_async(buf, h.a[root].ptr, bytes, s);
            mine = record(s);
        }
        hipEvent_t my_a = h.a[me_].ev;
        h.b[me_].ev = mine;
        h.barrier();
        if (me_ == root)
            for (int r = 0; r < h.n; ++r) if (r != root) wait_on(s, h.b[r].ev);
        destroy(my_a);
        pend_b_ = mine;
    }

    void allreduce_raw(const void* send, void* recv, size_t count, ScalarType t, ReduceOp op,
                       hipStream_t s) override {
        size_t mult;
        const char tc = type_char(t, mult);
        slate_error_if_msg(mult != 1 && op != ReduceOp::Sum, "complex max/min allreduce");
        const size_t bytes = count * scalar_size(t), elems = count * mult;
        Hub& h = *hub_;
        if (!h.dev) {
            h.a[me_].ptr = send;
            h.barrier();
            std::vector<const void*> in(h.n);
            for (int r = 0; r < h.n; ++r) in[r] = h.a[r].ptr;
            std::vector<char> acc(bytes);
            switch (tc) {
                case 'f': host_reduce<float>(reinterpret_cast<float*>(acc.data()), in, elems, op); break;
                case 'd': host_reduce<double>(reinterpret_cast<double*>(acc.data()), in, elems, op); break;
                case 'i': host_reduce<int32_t>(reinterpret_cast<int32_t*>(acc.data()), in, elems, op); break;
                case 'l': host_reduce<int64_t>(reinterpret_cast<int64_t*>(acc.data()), in, elems, op); break;
                default: host_reduce<int8_t>(reinterpret_cast<int8_t*>(acc.data()), in, elems, op); break;
            }
            h.barrier();                          // every rank has read every send buffer
            std::memcpy(recv, acc.data(), bytes);
            return;
        }
        if (h.n > 2 && bytes >= (size_t(1) << 20)) {
            allreduce_sliced(send, recv, elems, bytes / elems, tc, op, s);
            return;
        }
        h.a[me_] = {send, record(s)};
        h.barrier();
        destroy(pend_b_);
        char* tmp = static_cast<char*>(device::malloc_async(std::max<size_t>(size_t(h.n) * bytes, 1), s));
        for (int r = 0; r < h.n; ++r) {
            if (r != me_) wait_on(s, h.a[r].ev);
            device::memcpy_async(tmp + size_t(r) * bytes, h.a[r].ptr, bytes, s);
        }
        hipEvent_t my_a = h.a[me_].ev;
        hipEvent_t mine = record(s);
        h.b[me_].ev = mine;
        h.barrier();
        // recv may alias send: write only after every rank copied my send
        for (int r = 0; r < h.n; ++r) if (r != me_) wait_on(s, h.b[r].ev);
        slate_amd::dev::reduce_slabs(tc, op == ReduceOp::Sum ? 0 : op == ReduceOp::Max ? 1 : 2, recv, tmp, h.n,
                                     int64_t(elems), int64_t(elems), s);
        device::free_async(tmp, s);
        destroy(my_a);
        pend_b_ = mine;
    }

    /// Large all-reduce as reduce-scatter + all-gather: rank r pulls slice r
    /// of every rank's buffer, reduces it, and every rank then pulls the n
    /// reduced slices -- about 2 x bytes of peer traffic per rank instead of
    /// n x bytes for the all-to-all copy of the small-message path.
    void allreduce_sliced(const void* send, void* recv, size_t elems, size_t esize, char tc, ReduceOp op,
                          hipStream_t s) {
        Hub& h = *hub_;
        const int n = h.n;
        auto lo = [&](int r) { return elems * size_t(r) / size_t(n); };
        const size_t smax = (elems + n - 1) / n;                 // longest slice (elements)
        const size_t mine_lo = lo(me_), mine_len = lo(me_ + 1) - mine_lo;
        h.a[me_] = {send, record(s)};
        h.barrier();                                             // (1) every send buffer ready
        destroy(pend_b_);
        char* tmp = static_cast<char*>(device::malloc_async(std::max<size_t>((n + 1) * smax * esize, 1), s));
        char* red = tmp + size_t(n) * smax * esize;
        for (int r = 0; r < n; ++r) {
            if (r != me_) wait_on(s, h.a[r].ev);
            device::memcpy_async(tmp + size_t(r) * smax * esize,
                                 static_cast<const char*>(h.a[r].ptr) + mine_lo * esize, mine_len * esize, s);
        }
        if (mine_len > 0)
            slate_amd::dev::reduce_slabs(tc, op == ReduceOp::Sum ? 0 : op == ReduceOp::Max ? 1 : 2, red, tmp, n,
                                         int64_t(mine_len), int64_t(smax), s);
        hipEvent_t my_a = h.a[me_].ev;
        h.b[me_] = {red, record(s)};
        h.barrier();                                             // (2) every reduced slice published
        destroy(my_a);
        // recv may alias send: every rank's reads of my send finished before its slice event
        for (int r = 0; r < n; ++r) if (r != me_) wait_on(s, h.b[r].ev);
        for (int r = 0; r < n; ++r)
            device::memcpy_async(static_cast<char*>(recv) + lo(r) * esize, h.b[r].ptr, (lo(r + 1) - lo(r)) * esize,
                                 s);
        hipEvent_t my_b = h.b[me_].ev;
        hipEvent_t mine = record(s);
        h.c[me_] = {nullptr, mine};
        h.barrier();                                             // (3) every copy of the slices issued
        destroy(my_b);
        for (int r = 0; r < n; ++r) if (r != me_) wait_on(s, h.c[r].ev);
        device::free_async(tmp, s);                              // after the others read my slice
        pend_b_ = mine;
    }

    void allgather_raw(const void* send, void* recv, size_t count, ScalarType t, hipStream_t s) override {
        const size_t bytes = count * scalar_size(t);
        Hub& h = *hub_;
        char* out = static_cast<char*>(recv);
        if (!h.dev) {
            h.a[me_].ptr = send;
            h.barrier();
            for (int r = 0; r < h.n; ++r)
                if (out + size_t(r) * bytes != h.a[r].ptr) std::memmove(out + size_t(r) * bytes, h.a[r].ptr, bytes);
            h.barrier();
            return;
        }
        h.a[me_] = {send, record(s)};
        h.barrier();
        destroy(pend_b_);
        for (int r = 0; r < h.n; ++r) {
            if (r != me_) wait_on(s, h.a[r].ev);
            if (out + size_t(r) * bytes != h.a[r].ptr)
                device::memcpy_async(out + size_t(r) * bytes, h.a[r].ptr, bytes, s);
        }
        hipEvent_t my_a = h.a[me_].ev;
        hipEvent_t mine = record(s);
        h.b[me_].ev = mine;
        h.barrier();
        for (int r = 0; r < h.n; ++r) if (r != me_) wait_on(s, h.b[r].ev);
        destroy(my_a);
        pend_b_ = mine;
    }

    void send_raw(const void* buf, size_t count, ScalarType t, int peer, hipStream_t s) override {
        P2POp o{const_cast<void*>(buf), count * scalar_size(t), peer, true, s};
        if (in_group_) ops_.push_back(o);
        else run({o});
    }
    void recv_raw(void* buf, size_t count, ScalarType t, int peer, hipStream_t s) override {
        P2POp o{buf, count * scalar_size(t), peer, false, s};
        if (in_group_) ops_.push_back(o);
        else run({o});
    }
    void group_start() override { in_group_ = true; ops_.clear(); }
    void group_end() override {
        in_group_ = false;
        auto ops = std::move(ops_);
        ops_.clear();
        run(ops);
    }
    void barrier() override { hub_->barrier(); }

private:
    struct P2POp { void* buf; size_t bytes; int peer; bool send; hipStream_t s; };

    /// Post every send, then serve every receive (FIFO per (src, dst)), then
    /// wait until each posted send was consumed (blocking-send semantics).
    void run(std::vector<P2POp> const& ops) {
        Hub& h = *hub_;
        std::vector<std::pair<P2POp, std::shared_ptr<Hub::Msg>>> sent;
        for (auto const& o : ops) {
            if (!o.send) continue;
            auto msg = std::make_shared<Hub::Msg>();
            msg->ptr = o.buf;
            msg->bytes = o.bytes;
            msg->ev = h.dev ? record(o.s) : nullptr;
            {
                std::lock_guard<std::mutex> l(h.m);
                h.check();
                h.box[{me_, o.peer}].push_back(msg);
            }
            h.cv.notify_all();
            sent.emplace_back(o, msg);
        }
        for (auto const& o : ops) {
            if (o.send) continue;
            std::shared_ptr<Hub::Msg> msg;
            {
                std::unique_lock<std::mutex> l(h.m);
                auto& q = h.box[{o.peer, me_}];
                h.cv.wait(l, [&] { return !q.empty() || h.aborted; });
                h.check();
                msg = q.front();
                q.pop_front();
            }
            slate_error_if_msg(msg->bytes != o.bytes, "in-process recv: message size mismatch");
            hipEvent_t done = nullptr;
            if (h.dev) {
                wait_on(o.s, msg->ev);
                device::memcpy_async(o.buf, msg->ptr, o.bytes, o.s);
                done = record(o.s);
            } else {
                std::memcpy(o.buf, msg->ptr, o.bytes);
            }
            {
                std::lock_guard<std::mutex> l(h.m);
                msg->done = done;
                msg->completed = true;
            }
            h.cv.notify_all();
        }
        for (auto& sm : sent) {
            auto& msg = sm.second;
            {
                std::unique_lock<std::mutex> l(h.m);
                h.cv.wait(l, [&] { return msg->completed || h.aborted; });
                h.check();
            }
            if (h.dev) {
                wait_on(sm.first.s, msg->done);   // my buffer is free once the peer's copy is done
                destroy(msg->ev);
                destroy(msg->done);
            }
        }
    }

    std::shared_ptr<Hub> hub_;
    int me_;
    hipEvent_t pend_b_ = nullptr;   // my phase-B event of the previous collective
    bool in_group_ = false;
    std::vector<P2POp> ops_;
};

void enable_peer_access(std::vector<int> const& devs) {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return;
    for (int a : devs)
        for (int b : devs) {
            if (a == b) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) {
                // copies between a and b still work, staged by the runtime through
                // host memory -- far slower than xGMI: say so once
                static std::once_flag warned;
                std::call_once(warned, [&] {
                    std::fprintf(stderr, "slate: GPU %d cannot access GPU %d as a peer; in-process ranks "
                                 "exchange data through host staging (slow)\n", a, b);
                });
                continue;
            }
            (void)hipSetDevice(a);
            hipError_t e = hipDeviceEnablePeerAccess(b, 0);
            if (e == hipErrorPeerAccessAlreadyEnabled || e == hipSuccess) { (void)hipGetLastError(); continue; }
            (void)hipGetLastError();
            (void)hipSetDevice(cur);
            throw DeviceException(std::string("hipDeviceEnablePeerAccess(") + std::to_string(a) + " -> " +
                                      std::to_string(b) + "): " + hipGetErrorString(e),
                                  __func__, __FILE__, __LINE__);
        }
    (void)hipSetDevice(cur);
}

}  // namespace

std::vector<CommPtr> make_thread_comms(int n, bool device_mode) {
    slate_error_if_msg(n < 1, "make_thread_comms: n < 1");
    auto hub = std::make_shared<Hub>(n, device_mode);
    std::vector<CommPtr> v;
    for (int r = 0; r < n; ++r) v.push_back(std::make_shared<ThreadComm>(hub, r));
    return v;
}

void thread_comm_abort(Comm& c) {
    if (auto* t = dynamic_cast<ThreadComm*>(&c)) t->abort();
}

std::vector<GridPtr> make_thread_grids(int p, int q, GridOrder order, std::vector<int> const& devices) {
    const int n = p * q;
    const bool dev = !devices.empty();
    if (dev) {
        std::vector<int> u = devices;
        std::sort(u.begin(), u.end());
        u.erase(std::unique(u.begin(), u.end()), u.end());
        enable_peer_access(u);
    }
    auto world = make_thread_comms(n, dev);
    auto rank_of = [&](int r, int c) { return order == GridOrder::Col ? r + c * p : r * q + c; };
    // row comms (one hub per process row, rank = process column), column comms
    // (one hub per process column, rank = process row); plus the fast lanes
    std::vector<std::vector<CommPtr>> rows(p), cols(q), rows_f(p), cols_f(q);
    for (int r = 0; r < p; ++r) { rows[r] = make_thread_comms(q, dev); rows_f[r] = make_thread_comms(q, dev); }
    for (int c = 0; c < q; ++c) { cols[c] = make_thread_comms(p, dev); cols_f[c] = make_thread_comms(p, dev); }
    std::vector<GridPtr> grids(n);
    for (int r = 0; r < p; ++r)
        for (int c = 0; c < q; ++c) {
            const int w = rank_of(r, c);
            auto g = std::make_shared<Grid>(p, q, order, world[w], rows[r][c], cols[c][r]);
            g->set_fast(rows_f[r][c], cols_f[c][r]);
            grids[w] = g;
        }
    return grids;
}

void thread_grid_abort(Grid const& g) {
    for (CommPtr c : {g.world_ptr(), g.row_ptr(), g.col_ptr(), g.row_fast_ptr(), g.col_fast_ptr()})
        if (c) thread_comm_abort(*c);
}

void thread_grid_reset(Grid const& g) {
    for (CommPtr c : {g.world_ptr(), g.row_ptr(), g.col_ptr(), g.row_fast_ptr(), g.col_fast_ptr()})
        if (auto* t = c ? dynamic_cast<ThreadComm*>(c.get()) : nullptr) t->reset();
}

}  // namespace slate
