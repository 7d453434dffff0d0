#include "slate_amd/runtime.hh"
#include "slate_amd/trace.hh"

#include <mutex>

namespace slate {

namespace {
std::mutex g_lane_mtx;
bool g_lane_on = false;
std::vector<std::pair<std::string, int>> g_lane_log;
}  // namespace

void Sched::lane_log_enable(bool on) {
    std::lock_guard<std::mutex> l(g_lane_mtx);
    g_lane_on = on;
    g_lane_log.clear();
}

std::vector<std::pair<std::string, int>> Sched::lane_log_take() {
    std::lock_guard<std::mutex> l(g_lane_mtx);
    auto v = std::move(g_lane_log);
    g_lane_log.clear();
    return v;
}

Sched::Sched(Target target) : target_(target) {}

Sched::~Sched() {
    try { wait_all(); } catch (...) {}
    for (auto e : events_) device::event_put(e);
}

lb::Ctx Sched::ctx(int queue) const {
    if (target_ != Target::Devices) return lb::Ctx{target_, nullptr};
    return lb::Ctx{Target::Devices, device::queue(queue)};
}

void Sched::task(int queue, std::initializer_list<int64_t> in, std::initializer_list<int64_t> out, Fn fn) {
    task(queue, std::vector<int64_t>(in), std::vector<int64_t>(out), std::move(fn));
}

void Sched::task(int queue, std::vector<int64_t> const& in, std::vector<int64_t> const& out, Fn fn) {
    const bool lane = g_lane_on;
    if (target_ != Target::Devices) {
        if (lane) trace::task_label_begin();
        fn(ctx(queue));
        if (lane) {
            const char* l = trace::task_label_end();
            std::lock_guard<std::mutex> g(g_lane_mtx);
            g_lane_log.emplace_back(l ? l : "task", queue);
        }
        return;
    }
    hipStream_t s = device::queue(queue);
    used_[queue] = true;
    // RAW: wait for the last writer of every input and output token;
    // WAR: outputs also wait for all readers since that write.
    auto wait = [&](hipEvent_t e) { if (e) slate_hip_call(hipStreamWaitEvent(s, e, 0)); };
    for (int64_t t : in) wait(tokens_[t].writer);
    for (int64_t t : out) {
        auto& st = tokens_[t];
        wait(st.writer);
        for (auto e : st.readers) wait(e);
    }
    // tracing: one device span per task (timing events around its kernels),
    // labeled by the task's first trace::Block, on lane 100 + queue
    hipEvent_t ta = nullptr;
    if (trace::Trace::is_on() && hipEventCreate(&ta) == hipSuccess) {
        (void)hipEventRecord(ta, s);
        trace::task_label_begin();
    } else if (lane) {
        trace::task_label_begin();
    }
    fn(ctx(queue));
    if (!ta && lane) {
        const char* l = trace::task_label_end();
        std::lock_guard<std::mutex> g(g_lane_mtx);
        g_lane_log.emplace_back(l ? l : "task", queue);
    }
    if (ta) {
        const char* label = trace::task_label_end();
        if (lane) {
            std::lock_guard<std::mutex> g(g_lane_mtx);
            g_lane_log.emplace_back(label ? label : "task", queue);
        }
        hipEvent_t tb = nullptr;
        if (hipEventCreate(&tb) == hipSuccess) {
            (void)hipEventRecord(tb, s);
            trace::Trace::insert_device(label ? label : "task", queue, ta, tb);
        }
    }
    hipEvent_t e = device::event_get();
    events_.push_back(e);
    slate_hip_call(hipEventRecord(e, s));
    for (int64_t t : in) tokens_[t].readers.push_back(e);
    for (int64_t t : out) {
        auto& st = tokens_[t];
        st.writer = e;
        st.readers.clear();
    }
}

void Sched::wait_all() {
    if (target_ != Target::Devices) return;
    for (int q = 0; q < device::kNumQueues; ++q)
        if (used_[q]) slate_hip_call(hipStreamSynchronize(device::queue(q)));
}

}  // namespace slate
