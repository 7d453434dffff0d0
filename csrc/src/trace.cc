#include "slate_amd/trace.hh"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <cstdio>
#include <ctime>
#include <map>
#include <mutex>
#include <sstream>
#include <thread>

namespace slate {
namespace trace {

namespace {

struct PendingDev { std::string name; int queue; hipEvent_t a, b; };

struct State {
    std::mutex mtx;
    bool on = false;
    std::chrono::steady_clock::time_point origin = std::chrono::steady_clock::now();
    std::vector<Event> events;
    std::vector<PendingDev> pending;
    std::map<std::thread::id, int> lanes;
    std::string comment;
    hipEvent_t origin_event = nullptr;
    double origin_event_host = 0;
};

State& st() { static State* s = new State(); return *s; }

int lane_of_thread(State& s) {
    auto id = std::this_thread::get_id();
    auto it = s.lanes.find(id);
    if (it != s.lanes.end()) return it->second;
    int l = int(s.lanes.size());
    s.lanes[id] = l;
    return l;
}

void resolve_device(State& s) {
    if (s.pending.empty()) return;
    for (auto& p : s.pending) {
        float ms_a = 0, ms_b = 0;
        if (s.origin_event && hipEventSynchronize(p.b) == hipSuccess &&
            hipEventElapsedTime(&ms_a, s.origin_event, p.a) == hipSuccess &&
            hipEventElapsedTime(&ms_b, s.origin_event, p.b) == hipSuccess) {
            Event e{};
            std::strncpy(e.name, p.name.c_str(), sizeof(e.name) - 1);
            e.start = s.origin_event_host + ms_a * 1e-3;
            e.stop = s.origin_event_host + ms_b * 1e-3;
            e.lane = 100 + p.queue;
            s.events.push_back(e);
        }
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    s.pending.clear();
}

const char* color_for(const char* name) {
    static const char* palette[] = {"#e6194b", "#3cb44b", "#ffe119", "#4363d8", "#f58231", "#911eb4",
                                    "#46f0f0", "#f032e6", "#bcf60c", "#fabebe", "#008080", "#e6beff"};
    unsigned h = 0;
    for (const char* p = name; *p; ++p) h = h * 131 + unsigned(*p);
    return palette[h % 12];
}

}  // namespace

void Trace::on() { auto& s = st(); std::lock_guard<std::mutex> g(s.mtx); s.on = true; }
void Trace::off() { auto& s = st(); std::lock_guard<std::mutex> g(s.mtx); s.on = false; }
bool Trace::is_on() { return st().on; }

double Trace::now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - st().origin).count();
}

void Trace::insert(Event const& e) {
    auto& s = st();
    std::lock_guard<std::mutex> g(s.mtx);
    s.events.push_back(e);
}

void Trace::insert_device(const char* name, int queue, hipEvent_t a, hipEvent_t b) {
    auto& s = st();
    std::lock_guard<std::mutex> g(s.mtx);
    if (!s.origin_event) {
        // anchor device time: an event recorded now on the null stream
        if (hipEventCreate(&s.origin_event) == hipSuccess) {
            (void)hipEventRecord(s.origin_event, nullptr);
            (void)hipEventSynchronize(s.origin_event);
            s.origin_event_host = std::chrono::duration<double>(std::chrono::steady_clock::now() - s.origin).count();
        }
    }
    s.pending.push_back({name, queue, a, b});
}

void Trace::comment(std::string const& c) { auto& s = st(); std::lock_guard<std::mutex> g(s.mtx); s.comment = c; }

std::vector<Event> Trace::events() {
    auto& s = st();
    std::lock_guard<std::mutex> g(s.mtx);
    resolve_device(s);
    return s.events;
}

void Trace::clear() {
    auto& s = st();
    std::lock_guard<std::mutex> g(s.mtx);
    resolve_device(s);
    s.events.clear();
}

std::string Trace::finish(Comm* comm, std::string const& basename) {
    auto& s = st();
    std::vector<Event> mine;
    {
        std::lock_guard<std::mutex> g(s.mtx);
        resolve_device(s);
        mine = s.events;
    }
    int rank = comm ? comm->rank() : 0, size = comm ? comm->size() : 1;
    // gather counts then events (as raw bytes) to everyone (allgather), rank 0 writes
    std::vector<std::vector<Event>> all(size);
    if (size == 1) all[0] = mine;
    else {
        int64_t n = int64_t(mine.size());
        std::vector<int64_t> counts(size);
        comm->allgather(&n, counts.data(), 1, ScalarType::Int64, Loc::Host, nullptr);
        int64_t mx = *std::max_element(counts.begin(), counts.end());
        std::vector<Event> sendbuf(std::max<int64_t>(mx, 1));
        std::copy(mine.begin(), mine.end(), sendbuf.begin());
        std::vector<Event> recv(size_t(std::max<int64_t>(mx, 1)) * size);
        comm->allgather(sendbuf.data(), recv.data(), size_t(std::max<int64_t>(mx, 1)) * sizeof(Event),
                        ScalarType::Byte, Loc::Host, nullptr);
        for (int r = 0; r < size; ++r)
            all[r].assign(recv.begin() + size_t(r) * std::max<int64_t>(mx, 1),
                          recv.begin() + size_t(r) * std::max<int64_t>(mx, 1) + counts[r]);
    }
    if (rank != 0) return "";
    std::string base = basename.empty() ? "trace_" + std::to_string((long long)std::time(nullptr)) : basename;
    // Chrome trace JSON
    {
        FILE* f = std::fopen((base + ".json").c_str(), "w");
        if (f) {
            std::fprintf(f, "{\"traceEvents\":[\n");
            bool first = true;
            for (int r = 0; r < size; ++r)
                for (auto const& e : all[r]) {
                    std::fprintf(f, "%s{\"name\":\"%s\",\"ph\":\"X\",\"pid\":%d,\"tid\":%d,\"ts\":%.3f,\"dur\":%.3f}",
                                 first ? "" : ",\n", e.name, r, e.lane, e.start * 1e6, (e.stop - e.start) * 1e6);
                    first = false;
                }
            std::fprintf(f, "\n],\"otherData\":{\"comment\":\"%s\"}}\n", s.comment.c_str());
            std::fclose(f);
        }
    }
    // SVG timeline (one row per (rank, lane))
    {
        double t0 = 1e300, t1 = -1e300;
        std::map<std::pair<int, int>, int> rows;
        for (int r = 0; r < size; ++r)
            for (auto const& e : all[r]) {
                t0 = std::min(t0, e.start); t1 = std::max(t1, e.stop);
                rows.emplace(std::make_pair(r, e.lane), 0);
            }
        int ri = 0;
        for (auto& kv : rows) kv.second = ri++;
        double W = 1600, H = 20.0 * std::max(1, ri) + 60, span = std::max(t1 - t0, 1e-9);
        FILE* f = std::fopen((base + ".svg").c_str(), "w");
        if (f) {
            std::fprintf(f, "<svg xmlns=\"http://www.w3.org/2000/svg\" width=\"%.0f\" height=\"%.0f\">\n", W + 200, H);
            for (auto& kv : rows)
                std::fprintf(f, "<text x=\"0\" y=\"%d\" font-size=\"10\">rank %d %s %d</text>\n", 20 * kv.second + 14,
                             kv.first.first, kv.first.second >= 100 ? "queue" : "thread",
                             kv.first.second >= 100 ? kv.first.second - 100 : kv.first.second);
            for (int r = 0; r < size; ++r)
                for (auto const& e : all[r]) {
                    int row = rows[std::make_pair(r, e.lane)];
                    double x = 150 + (e.start - t0) / span * W, w = std::max(0.5, (e.stop - e.start) / span * W);
                    std::fprintf(f, "<rect x=\"%.2f\" y=\"%d\" width=\"%.2f\" height=\"16\" fill=\"%s\"><title>%s %.3f ms</title></rect>\n",
                                 x, 20 * row + 2, w, color_for(e.name), e.name, (e.stop - e.start) * 1e3);
                }
            std::fprintf(f, "<text x=\"150\" y=\"%.0f\" font-size=\"12\">span %.3f ms. %s</text>\n</svg>\n",
                         H - 10, span * 1e3, s.comment.c_str());
            std::fclose(f);
        }
    }
    return base;
}

namespace {
/// SLATE_DEBUG_CALLS=1: every traced routine logs entry/exit to stderr with
/// the world rank (reference Debug.cc-style diagnostics; finds the routine a
/// multi-rank hang is stuck in).
bool debug_calls() {
    static bool on = [] { const char* e = std::getenv("SLATE_DEBUG_CALLS"); return e && *e && *e != '0'; }();
    return on;
}
int debug_rank() {
    const char* e = std::getenv("RANK");
    return e ? std::atoi(e) : 0;
}
}  // namespace

namespace {
thread_local const char* t_task_label = nullptr;
thread_local bool t_task_open = false;
}  // namespace

void task_label_begin() { t_task_open = true; t_task_label = nullptr; }
const char* task_label_end() { t_task_open = false; const char* l = t_task_label; t_task_label = nullptr; return l; }

Block::Block(const char* name) : name_(name), start_(0), active_(Trace::is_on()) {
    if (t_task_open && !t_task_label) t_task_label = name;   // first span inside a Sched task labels it
    if (active_) start_ = Trace::now();
    if (debug_calls()) std::fprintf(stderr, "[rank %d] > %s\n", debug_rank(), name);
}

Block::~Block() { end(); }

void Block::end() {
    if (ended_) return;
    ended_ = true;
    if (debug_calls()) std::fprintf(stderr, "[rank %d] < %s\n", debug_rank(), name_);
    if (!active_) return;
    Event e{};
    std::strncpy(e.name, name_, sizeof(e.name) - 1);
    e.start = start_;
    e.stop = Trace::now();
    {
        auto& s = st();
        std::lock_guard<std::mutex> g(s.mtx);
        e.lane = lane_of_thread(s);
        s.events.push_back(e);
    }
}

DeviceBlock::DeviceBlock(const char* name, int queue) : name_(name), queue_(queue) {
    if (!Trace::is_on()) return;
    if (hipEventCreate(&start_) != hipSuccess) { start_ = nullptr; return; }
    (void)hipEventRecord(start_, device::queue(queue_));
}

DeviceBlock::~DeviceBlock() {
    if (!start_) return;
    hipEvent_t stop;
    if (hipEventCreate(&stop) != hipSuccess) return;
    (void)hipEventRecord(stop, device::queue(queue_));
    Trace::insert_device(name_, queue_, start_, stop);
}

}  // namespace trace
}  // namespace slate
