// Tracing (reference include/slate/internal/Trace.hh, src/auxiliary/Trace.cc:
// RAII trace::Block host spans gathered to rank 0 and written as an SVG).
//
// Here: host spans (RAII Block) plus optional DEVICE spans measured with
// timing hipEvents on the queue that ran the work, gathered to rank 0 over
// the world communicator and written as Chrome-trace JSON (chrome://tracing /
// Perfetto) and as an SVG timeline like the reference's.
#pragma once

#include "comm.hh"

#include <string>
#include <vector>

namespace slate {
namespace trace {

struct Event {
    char name[32];
    double start, stop;   // seconds since trace origin
    int lane;             // host thread (0..) or 100 + device queue index
};

class Trace {
public:
    static void on();
    static void off();
    static bool is_on();
    static void insert(Event const& e);
    static double now();
    /// Record a device span between two timing events on `queue` (resolved at finish).
    static void insert_device(const char* name, int queue, hipEvent_t start, hipEvent_t stop);
    static void comment(std::string const& c);
    /// Gather all ranks' events to rank 0 and write `<basename>.json` and
    /// `<basename>.svg`.  Collective over `comm` (may be null: local only).
    static std::string finish(Comm* comm = nullptr, std::string const& basename = "");
    static std::vector<Event> events();
    static void clear();
};

/// Label of the Sched task being enqueued on this thread: the name of the
/// first trace::Block opened between task_label_begin() and task_label_end()
/// (null if none) -- the runtime's device spans of a task carry it.
void task_label_begin();
const char* task_label_end();

/// RAII host span.
class Block {
public:
    explicit Block(const char* name);
    ~Block();
    /// close the span before the end of the scope (once)
    void end();
private:
    const char* name_;
    double start_;
    bool active_;
    bool ended_ = false;
};

/// RAII device span on a HIP queue (records timing events when tracing is on).
class DeviceBlock {
public:
    DeviceBlock(const char* name, int queue);
    ~DeviceBlock();
private:
    const char* name_;
    int queue_;
    hipEvent_t start_ = nullptr;
};

}  // namespace trace
}  // namespace slate
