// Native host transport over TCP sockets, and the C++ process-grid bootstrap.
//
// The reference builds on MPI (MPI_Init_thread in
// test/test.cc:593-599) and ships single-rank MPI stubs for builds without it
// (src/stubs/mpi_stubs.cc).  There is no MPI on the MI355X node; production
// multi-GPU traffic goes over RCCL/xGMI (rccl_comm.cc).  This file provides
// the two things MPI gave a standalone C++ program besides the data plane:
//
//  * a launcher-agnostic rendezvous: ranks find each other from the
//    torchrun-style environment (RANK, WORLD_SIZE, MASTER_ADDR, and
//    SLATE_MASTER_PORT or MASTER_PORT+17), build a full socket mesh, and
//    exchange the RCCL unique id over it;
//  * a host transport (TcpComm, a HostComm) for CPU-only runs and for the
//    control plane: bcast / allreduce / allgather / send / recv on host
//    buffers, with sub-communicators from split().  Device buffers are
//    staged by the Comm wrappers (comm.cc), like non-GPU-aware MPI.
//
// One receiver thread per peer drains every incoming frame into per-
// communicator mailboxes, so sends never block on the peer's progress and
// messages of different communicators sharing a socket cannot deadlock.
#include "slate_amd/init.hh"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <complex>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

namespace slate {

namespace {

[[noreturn]] void sys_fail(std::string const& what) {
    throw CommException(what + ": " + std::strerror(errno), __func__, __FILE__, __LINE__);
}

void write_all(int fd, const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    while (n > 0) {
        ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
        if (w < 0) { if (errno == EINTR) continue; sys_fail("tcp send"); }
        c += w; n -= size_t(w);
    }
}

bool read_all(int fd, void* p, size_t n) {
    char* c = static_cast<char*>(p);
    while (n > 0) {
        ssize_t r = ::recv(fd, c, n, 0);
        if (r == 0) return false;
        if (r < 0) { if (errno == EINTR) continue; return false; }
        c += r; n -= size_t(r);
    }
    return true;
}

/// receive timeout on a socket (0 = none): a stray connection that sends
/// nothing cannot block a rendezvous / mesh accept forever
void set_rcv_timeout(int fd, double seconds) {
    timeval tv{};
    tv.tv_sec = time_t(seconds);
    tv.tv_usec = suseconds_t((seconds - double(tv.tv_sec)) * 1e6);
    ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
}

int env_int(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return e && *e ? std::atoi(e) : dflt;
}

std::string env_str(const char* name, const char* dflt) {
    const char* e = std::getenv(name);
    return e && *e ? std::string(e) : std::string(dflt);
}

/// True when every rank reaches the master over loopback (single-node jobs
/// launched with MASTER_ADDR=127.0.0.1 / localhost): the listeners are then
/// bound to 127.0.0.1 only instead of every interface.
bool loopback_job(std::string const& master) {
    return master == "localhost" || master.rfind("127.", 0) == 0;
}

/// Per-job handshake token: SLATE_JOB_TOKEN if set, else a hash of the
/// launcher environment every rank of the job shares (torchrun run id,
/// master address/port, world size).  Peers presenting another token are
/// rejected, so a stray connection cannot pose as a rank of this job.
uint64_t job_token() {
    std::string k = env_str("SLATE_JOB_TOKEN", "");
    if (k.empty())
        k = env_str("TORCHELASTIC_RUN_ID", "") + "|" + env_str("MASTER_ADDR", "127.0.0.1") + "|" +
            env_str("MASTER_PORT", "") + "|" + env_str("SLATE_MASTER_PORT", "") + "|" + env_str("WORLD_SIZE", "1");
    uint64_t h = 1469598103934665603ull;   // FNV-1a
    for (unsigned char c : k) { h ^= c; h *= 1099511628211ull; }
    return h;
}

int listen_on(int port, int& bound_port, bool loopback) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) sys_fail("socket");
    int one = 1;
    ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(loopback ? INADDR_LOOPBACK : INADDR_ANY);
    a.sin_port = htons(uint16_t(port));
    if (::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) < 0) sys_fail("bind port " + std::to_string(port));
    if (::listen(fd, 256) < 0) sys_fail("listen");
    socklen_t len = sizeof(a);
    ::getsockname(fd, reinterpret_cast<sockaddr*>(&a), &len);
    bound_port = ntohs(a.sin_port);
    return fd;
}

int connect_to(std::string const& host, int port, double timeout_s) {
    auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        addrinfo hints{}, *res = nullptr;
        hints.ai_family = AF_INET;
        hints.ai_socktype = SOCK_STREAM;
        if (::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) == 0 && res) {
            int fd = ::socket(AF_INET, SOCK_STREAM, 0);
            if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
                ::freeaddrinfo(res);
                int one = 1;
                ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
                return fd;
            }
            if (fd >= 0) ::close(fd);
            ::freeaddrinfo(res);
        }
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (dt > timeout_s)
            throw CommException("tcp rendezvous: cannot connect to " + host + ":" + std::to_string(port),
                                __func__, __FILE__, __LINE__);
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
}

//------------------------------------------------------------------------------
/// Full socket mesh between all ranks of the job + per-communicator mailboxes.
class TcpTransport {
public:
    TcpTransport(int rank, int size) : rank_(rank), size_(size), peers_(size) {}
    ~TcpTransport() {
        stop_ = true;
        for (auto& p : peers_)
            if (p.fd >= 0) ::shutdown(p.fd, SHUT_RDWR);
        for (auto& p : peers_)
            if (p.th.joinable()) p.th.join();
        for (auto& p : peers_)
            if (p.fd >= 0) ::close(p.fd);
    }

    int rank() const { return rank_; }
    int size() const { return size_; }

    void connect_mesh(std::string const& master, int master_port, double timeout_s) {
        if (size_ == 1) return;
        int my_port = 0;
        const bool lo = loopback_job(master);
        const uint64_t token = job_token();
        int lfd = listen_on(0, my_port, lo);
        // rendezvous at rank 0: gather (ip, port) of every rank, broadcast table
        std::vector<uint32_t> ips(size_, 0);
        std::vector<int32_t> ports(size_, 0);
        if (rank_ == 0) {
            int rport = 0;
            int rfd = listen_on(master_port, rport, lo);
            ports[0] = my_port;
            ips[0] = 0;  // peers reach rank 0 through `master`
            std::vector<int> fds;
            std::vector<char> seen(size_, 0);
            while (int(fds.size()) < size_ - 1) {
                sockaddr_in a{};
                socklen_t len = sizeof(a);
                int fd = ::accept(rfd, reinterpret_cast<sockaddr*>(&a), &len);
                if (fd < 0) sys_fail("accept (rendezvous)");
                set_rcv_timeout(fd, std::min(timeout_s, 10.0));
                Hello h{};
                // wrong token, bad or duplicate rank: drop the connection
                if (!read_all(fd, &h, sizeof(h)) || h.token != token || h.rank <= 0 || h.rank >= size_ ||
                    seen[h.rank]) {
                    ::close(fd);
                    continue;
                }
                set_rcv_timeout(fd, 0);
                seen[h.rank] = 1;
                ips[h.rank] = a.sin_addr.s_addr;
                ports[h.rank] = h.port;
                fds.push_back(fd);
            }
            for (int fd : fds) {
                write_all(fd, ips.data(), ips.size() * sizeof(uint32_t));
                write_all(fd, ports.data(), ports.size() * sizeof(int32_t));
                ::close(fd);
            }
            ::close(rfd);
        } else {
            int fd = connect_to(master, master_port, timeout_s);
            Hello h{token, rank_, my_port};
            write_all(fd, &h, sizeof(h));
            if (!read_all(fd, ips.data(), ips.size() * sizeof(uint32_t)) ||
                !read_all(fd, ports.data(), ports.size() * sizeof(int32_t)))
                sys_fail("rendezvous table");
            ::close(fd);
        }
        // mesh: connect to lower ranks, accept higher ranks
        for (int j = 0; j < rank_; ++j) {
            std::string host = master;
            if (j != 0) {
                char buf[INET_ADDRSTRLEN];
                in_addr ia{};
                ia.s_addr = ips[j];
                host = ::inet_ntop(AF_INET, &ia, buf, sizeof(buf));
            }
            int fd = connect_to(host, ports[j], timeout_s);
            Hello h{token, rank_, 0};
            write_all(fd, &h, sizeof(h));
            peers_[j].fd = fd;
        }
        for (int n = rank_ + 1; n < size_;) {
            int fd = ::accept(lfd, nullptr, nullptr);
            if (fd < 0) sys_fail("accept (mesh)");
            int one = 1;
            ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
            set_rcv_timeout(fd, std::min(timeout_s, 10.0));
            Hello h{};
            if (!read_all(fd, &h, sizeof(h)) || h.token != token || h.rank <= rank_ || h.rank >= size_ ||
                peers_[h.rank].fd >= 0) {
                ::close(fd);   // not a peer of this job (or a duplicate rank)
                continue;
            }
            set_rcv_timeout(fd, 0);   // the receiver thread blocks for the job's lifetime
            peers_[h.rank].fd = fd;
            ++n;
        }
        ::close(lfd);
        for (int j = 0; j < size_; ++j)
            if (j != rank_) peers_[j].th = std::thread([this, j] { receiver(j); });
    }

    void send(uint64_t comm_id, int peer, const void* buf, size_t bytes) {
        slate_error_if_msg(peer == rank_, "tcp send to self");
        Peer& p = peers_[peer];
        uint64_t hdr[2] = {comm_id, uint64_t(bytes)};
        std::lock_guard<std::mutex> l(p.wmtx);
        write_all(p.fd, hdr, sizeof(hdr));
        if (bytes) write_all(p.fd, buf, bytes);
    }

    void recv(uint64_t comm_id, int peer, void* buf, size_t bytes) {
        slate_error_if_msg(peer == rank_, "tcp recv from self");
        Peer& p = peers_[peer];
        std::vector<char> msg;
        {
            std::unique_lock<std::mutex> l(p.mmtx);
            p.cv.wait(l, [&] { return p.dead || !p.box[comm_id].empty(); });
            auto& q = p.box[comm_id];
            if (q.empty())
                throw CommException("tcp: peer " + std::to_string(peer) + " closed the connection",
                                    __func__, __FILE__, __LINE__);
            msg = std::move(q.front());
            q.pop_front();
        }
        slate_error_if_msg(msg.size() != bytes, "tcp recv: message size mismatch (" + std::to_string(msg.size()) +
                                                " vs " + std::to_string(bytes) + ")");
        if (bytes) std::memcpy(buf, msg.data(), bytes);
    }

    uint64_t new_comm_id(uint64_t parent, int color) {
        // deterministic across the members of a split: same parent, same
        // per-parent split counter, same color
        std::lock_guard<std::mutex> l(idmtx_);
        uint64_t n = ++splits_[parent];
        uint64_t h = parent * 0x9E3779B97F4A7C15ull ^ (n << 32) ^ uint64_t(uint32_t(color) + 1);
        h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 32;
        return h | 1;  // 0 is reserved for the world communicator
    }

private:
    /// Rendezvous / mesh handshake: job token, sender rank, listening port.
    struct Hello {
        uint64_t token;
        int32_t rank;
        int32_t port;
    };
    struct Peer {
        int fd = -1;
        std::thread th;
        std::mutex wmtx, mmtx;
        std::condition_variable cv;
        std::map<uint64_t, std::deque<std::vector<char>>> box;
        bool dead = false;
    };

    void receiver(int j) {
        Peer& p = peers_[j];
        for (;;) {
            uint64_t hdr[2];
            if (!read_all(p.fd, hdr, sizeof(hdr))) break;
            std::vector<char> msg(hdr[1]);
            if (hdr[1] && !read_all(p.fd, msg.data(), hdr[1])) break;
            std::lock_guard<std::mutex> l(p.mmtx);
            p.box[hdr[0]].push_back(std::move(msg));
            p.cv.notify_all();
        }
        std::lock_guard<std::mutex> l(p.mmtx);
        p.dead = true;
        p.cv.notify_all();
    }

    int rank_, size_;
    std::vector<Peer> peers_;
    bool stop_ = false;
    std::mutex idmtx_;
    std::map<uint64_t, uint64_t> splits_;
};

template <typename T>
void reduce_into(T* acc, const T* x, size_t n, ReduceOp op) {
    for (size_t i = 0; i < n; ++i) {
        if (op == ReduceOp::Sum) acc[i] += x[i];
        else if constexpr (!is_complex_v<T>) {
            if (op == ReduceOp::Max) acc[i] = std::max(acc[i], x[i]);
            else acc[i] = std::min(acc[i], x[i]);
        }
    }
}

void reduce_typed(void* acc, const void* x, size_t count, ScalarType t, ReduceOp op) {
    switch (t) {
        case ScalarType::Int32: reduce_into((int32_t*)acc, (const int32_t*)x, count, op); break;
        case ScalarType::Int64: reduce_into((int64_t*)acc, (const int64_t*)x, count, op); break;
        case ScalarType::Float32: reduce_into((float*)acc, (const float*)x, count, op); break;
        case ScalarType::Float64: reduce_into((double*)acc, (const double*)x, count, op); break;
        case ScalarType::Complex64:
            slate_error_if_msg(op != ReduceOp::Sum, "complex max/min allreduce");
            reduce_into((std::complex<float>*)acc, (const std::complex<float>*)x, count, op); break;
        case ScalarType::Complex128:
            slate_error_if_msg(op != ReduceOp::Sum, "complex max/min allreduce");
            reduce_into((std::complex<double>*)acc, (const std::complex<double>*)x, count, op); break;
        case ScalarType::Byte: reduce_into((uint8_t*)acc, (const uint8_t*)x, count, op); break;
    }
}

//------------------------------------------------------------------------------
class TcpComm : public HostComm {
public:
    TcpComm(std::shared_ptr<TcpTransport> t, uint64_t id, std::vector<int> members)
        : t_(std::move(t)), id_(id), members_(std::move(members)) {
        auto it = std::find(members_.begin(), members_.end(), t_->rank());
        slate_error_if_msg(it == members_.end(), "TcpComm: this rank is not a member");
        me_ = int(it - members_.begin());
    }
    int rank() const override { return me_; }
    int size() const override { return int(members_.size()); }
    std::string name() const override { return "tcp"; }

    void bcast_raw(void* buf, size_t count, ScalarType t, int root, hipStream_t) override {
        size_t bytes = count * scalar_size(t);
        if (me_ == root) {
            for (int r = 0; r < size(); ++r)
                if (r != root) t_->send(id_, members_[r], buf, bytes);
        } else {
            t_->recv(id_, members_[root], buf, bytes);
        }
    }
    void allreduce_raw(const void* send, void* recv, size_t count, ScalarType t, ReduceOp op,
                       hipStream_t) override {
        size_t bytes = count * scalar_size(t);
        if (send != recv) std::memmove(recv, send, bytes);
        if (me_ == 0) {
            std::vector<char> tmp(bytes);
            for (int r = 1; r < size(); ++r) {
                t_->recv(id_, members_[r], tmp.data(), bytes);
                reduce_typed(recv, tmp.data(), count, t, op);
            }
        } else {
            t_->send(id_, members_[0], recv, bytes);
        }
        bcast_raw(recv, count, t, 0, nullptr);
    }
    void allgather_raw(const void* send, void* recv, size_t count, ScalarType t, hipStream_t) override {
        size_t bytes = count * scalar_size(t);
        char* out = static_cast<char*>(recv);
        std::memmove(out + size_t(me_) * bytes, send, bytes);
        for (int r = 0; r < size(); ++r)
            if (r != me_) t_->send(id_, members_[r], send, bytes);
        for (int r = 0; r < size(); ++r)
            if (r != me_) t_->recv(id_, members_[r], out + size_t(r) * bytes, bytes);
    }
    void send_raw(const void* buf, size_t count, ScalarType t, int peer, hipStream_t) override {
        t_->send(id_, members_.at(peer), buf, count * scalar_size(t));
    }
    void recv_raw(void* buf, size_t count, ScalarType t, int peer, hipStream_t) override {
        t_->recv(id_, members_.at(peer), buf, count * scalar_size(t));
    }
    void barrier() override {
        int32_t one = 1;
        allreduce_raw(&one, &one, 1, ScalarType::Int32, ReduceOp::Sum, nullptr);
    }

    std::shared_ptr<TcpComm> split(int color, int key) {
        int32_t mine[2] = {color, key};
        std::vector<int32_t> all(2 * size());
        allgather_raw(mine, all.data(), 2, ScalarType::Int32, nullptr);
        std::vector<std::pair<int, int>> sel;  // (key, member index)
        for (int r = 0; r < size(); ++r)
            if (all[2 * r] == color) sel.push_back({all[2 * r + 1], r});
        std::stable_sort(sel.begin(), sel.end());
        std::vector<int> mem;
        for (auto& s : sel) mem.push_back(members_[s.second]);
        uint64_t nid = t_->new_comm_id(id_, color);
        return std::make_shared<TcpComm>(t_, nid, mem);
    }

private:
    std::shared_ptr<TcpTransport> t_;
    uint64_t id_;
    std::vector<int> members_;
    int me_ = 0;
};

std::mutex g_init_mtx;
std::shared_ptr<TcpComm> g_tcp_world;

}  // namespace

//------------------------------------------------------------------------------
int env_world_rank() { return env_int("RANK", 0); }
int env_world_size() { return env_int("WORLD_SIZE", 1); }

CommPtr make_tcp_world(double timeout_s) {
    std::lock_guard<std::mutex> l(g_init_mtx);
    if (g_tcp_world) return g_tcp_world;
    int rank = env_world_rank(), size = env_world_size();
    slate_error_if_msg(size < 1 || rank < 0 || rank >= size, "RANK / WORLD_SIZE environment is inconsistent");
    auto t = std::make_shared<TcpTransport>(rank, size);
    std::string master = env_str("MASTER_ADDR", "127.0.0.1");
    int port = env_int("SLATE_MASTER_PORT", env_int("MASTER_PORT", 29500) + 17);
    t->connect_mesh(master, port, timeout_s);
    std::vector<int> all(size);
    for (int r = 0; r < size; ++r) all[r] = r;
    g_tcp_world = std::make_shared<TcpComm>(t, 0, all);
    return g_tcp_world;
}

CommPtr tcp_split(CommPtr const& parent, int color, int key) {
    auto* p = dynamic_cast<TcpComm*>(parent.get());
    slate_error_if_msg(!p, "tcp_split: parent is not a TCP communicator");
    return p->split(color, key);
}

GridPtr init_grid(int p, int q, GridOrder order, std::string transport) {
    int n = env_world_size(), rank = env_world_rank();
    if (p <= 0 || q <= 0) {
        p = 1;
        for (int d = 1; d * d <= n; ++d)
            if (n % d == 0) p = d;
        q = n / p;
    }
    slate_error_if_msg(p * q != n, "init_grid: p*q must equal WORLD_SIZE");
    if (n == 1) {
        set_default_grid(Grid::self());
        return Grid::self();
    }
    if (device::available()) device::set_device(env_int("LOCAL_RANK", rank) % std::max(1, device::count()));
    if (transport == "auto") {
        std::string e = env_str("SLATE_COMM", "");
        transport = (device::available() && e != "host") ? "rccl" : "tcp";
    }
    CommPtr tcp = make_tcp_world();
    int myrow = order == GridOrder::Col ? rank % p : rank / q;
    int mycol = order == GridOrder::Col ? rank / p : rank % q;
    CommPtr world, row, col, rowf, colf;
    if (transport == "rccl") {
        std::string uid(128, '\0');
        if (rank == 0) uid = rccl_unique_id();
        uid.resize(128);
        tcp->bcast_raw(uid.data(), uid.size(), ScalarType::Byte, 0, nullptr);
        world = make_rccl_comm(uid, n, rank);
        row = rccl_split(world, myrow, mycol);
        col = rccl_split(world, p + mycol, myrow);
        // critical-path duplicates (Grid::row_fast / col_fast)
        rowf = rccl_split(world, myrow, mycol);
        colf = rccl_split(world, p + mycol, myrow);
    } else {
        slate_error_if_msg(transport != "tcp", "init_grid: transport must be auto, rccl or tcp");
        world = tcp;
        row = tcp_split(tcp, myrow, mycol);
        col = tcp_split(tcp, p + mycol, myrow);
    }
    auto g = std::make_shared<Grid>(p, q, order, world, row, col);
    if (rowf && std::getenv("SLATE_FAST_LANE") == nullptr) g->set_fast(rowf, colf);
    else if (rowf && std::atoi(std::getenv("SLATE_FAST_LANE")) != 0) g->set_fast(rowf, colf);
    set_default_grid(g);
    return g;
}

void finalize() {
    if (auto g = default_grid(); g && g->size() > 1) g->world().barrier();
    set_default_grid(Grid::self());
    std::lock_guard<std::mutex> l(g_init_mtx);
    g_tcp_world.reset();
}

}  // namespace slate
