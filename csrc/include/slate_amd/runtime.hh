// Dependency-DAG runtime over HIP streams.
//
// Reference: every driver builds an OpenMP task DAG (#pragma omp task
// depend(in/inout: column[k]) priority(p), src/potrf.cc:84-195,
// src/getrf.cc:82-237) and each internal op ends with queue->sync()
// (internal_gemm.cc:510), so the host blocks per op.
//
// Here a driver declares tasks with data tokens; a task is ENQUEUED on one of
// the per-process HIP queues after hipStreamWaitEvent on the events of the
// tasks it depends on (RAW, WAR and WAW tracked per token), and records an
// event for its successors.  The host never waits inside a factorization;
// lookahead falls out of putting the panel and lookahead columns on their own
// (high-priority) queues.  On host targets tasks simply run in program order.
#pragma once

#include "local_blas.hh"

#include <functional>
#include <initializer_list>
#include <map>
#include <string>
#include <utility>
#include <vector>

namespace slate {

class Sched {
public:
    explicit Sched(Target target);
    ~Sched();
    Sched(Sched const&) = delete;
    Sched& operator=(Sched const&) = delete;

    /// Queue indices: 0 trailing update, 1 panel (high priority), 2.. lookahead,
    /// device::kCommQueue communication.
    using Fn = std::function<void(lb::Ctx const&)>;
    void task(int queue, std::initializer_list<int64_t> in, std::initializer_list<int64_t> out, Fn fn);
    void task(int queue, std::vector<int64_t> const& in, std::vector<int64_t> const& out, Fn fn);

    /// Block the host until every enqueued task finished.
    void wait_all();
    lb::Ctx ctx(int queue) const;
    Target target() const { return target_; }
    bool device() const { return target_ == Target::Devices; }

    /// Lane log (tests / diagnostics): when enabled, every task appends
    /// (label of its first trace::Block, queue index) in enqueue order, on
    /// host targets too -- pins which queue (and so which communication
    /// lane) each critical-path and bulk task is issued on.
    static void lane_log_enable(bool on);
    static std::vector<std::pair<std::string, int>> lane_log_take();

    /// Token helpers for common dependency names.
    static int64_t col(int64_t k)  { return 1000000 + k; }
    static int64_t row(int64_t k)  { return 2000000 + k; }
    static int64_t bcast(int64_t k){ return 3000000 + k; }
    static int64_t work(int64_t k) { return 4000000 + k; }
    static int64_t tok(int64_t kind, int64_t k) { return kind * 1000000 + k; }

private:
    struct TokState {
        hipEvent_t writer = nullptr;
        std::vector<hipEvent_t> readers;
    };
    Target target_;
    std::map<int64_t, TokState> tokens_;
    std::vector<hipEvent_t> events_;
    bool used_[device::kNumQueues] = {};
};

}  // namespace slate
