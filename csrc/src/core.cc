// Version, timers and enum string conversions (reference src/version.cc,
// src/core/types.cc:23).
#include "slate_amd/util.hh"
#include "slate_amd/enums.hh"
#include "slate_amd/exception.hh"

#include <algorithm>
#include <cctype>
#include <mutex>

#ifndef SLATE_AMD_VERSION
#define SLATE_AMD_VERSION "2026.10.0"
#endif

namespace slate {

std::map<std::string, double>& timers() {
    static std::map<std::string, double>* t = new std::map<std::string, double>();
    return *t;
}

const char* version() { return SLATE_AMD_VERSION; }
const char* id() { return "slate_d35_amd gfx950"; }

const char* to_string(Target t) {
    switch (t) {
        case Target::Host: return "host";
        case Target::HostTask: return "task";
        case Target::HostNest: return "nest";
        case Target::HostBatch: return "batch";
        case Target::Devices: return "devices";
    }
    return "?";
}
const char* to_string(Op v) { return v == Op::NoTrans ? "notrans" : v == Op::Trans ? "trans" : "conjtrans"; }
const char* to_string(Uplo v) { return v == Uplo::Lower ? "lower" : v == Uplo::Upper ? "upper" : "general"; }
const char* to_string(Norm v) {
    switch (v) {
        case Norm::One: return "1"; case Norm::Two: return "2"; case Norm::Inf: return "inf";
        case Norm::Fro: return "fro"; case Norm::Max: return "max";
    }
    return "?";
}

Target str2target(const std::string& s_) {
    std::string s = s_;
    std::transform(s.begin(), s.end(), s.begin(), ::tolower);
    if (s == "h" || s == "host") return Target::Host;
    if (s == "t" || s == "task" || s == "hosttask") return Target::HostTask;
    if (s == "n" || s == "nest" || s == "hostnest") return Target::HostNest;
    if (s == "b" || s == "batch" || s == "hostbatch") return Target::HostBatch;
    if (s == "d" || s == "dev" || s == "device" || s == "devices") return Target::Devices;
    throw Exception("unknown target: " + s_);
}

Norm str2norm(const std::string& s_) {
    std::string s = s_;
    std::transform(s.begin(), s.end(), s.begin(), ::tolower);
    if (s == "1" || s == "o" || s == "one") return Norm::One;
    if (s == "2" || s == "two") return Norm::Two;
    if (s == "i" || s == "inf") return Norm::Inf;
    if (s == "f" || s == "fro") return Norm::Fro;
    if (s == "m" || s == "max") return Norm::Max;
    throw Exception("unknown norm: " + s_);
}

}  // namespace slate
