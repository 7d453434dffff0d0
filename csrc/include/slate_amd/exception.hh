// Exceptions and assertion macros (reference include/slate/Exception.hh:16-122).
#pragma once

#include <exception>
#include <string>
#include <cstdio>

namespace slate {

class Exception : public std::exception {
public:
    Exception() : msg_() {}
    explicit Exception(std::string const& msg) : msg_(msg) {}
    Exception(std::string const& msg, const char* func, const char* file, int line)
        : msg_(msg + " in " + func + " at " + file + ":" + std::to_string(line)) {}
    const char* what() const noexcept override { return msg_.c_str(); }
protected:
    std::string msg_;
};

class NotImplemented : public Exception {
public:
    NotImplemented(std::string const& msg, const char* func, const char* file, int line)
        : Exception(std::string("not yet implemented: ") + msg, func, file, line) {}
};

class DeviceException : public Exception {
public:
    DeviceException(std::string const& msg, const char* func, const char* file, int line)
        : Exception(std::string("HIP error: ") + msg, func, file, line) {}
};

class CommException : public Exception {
public:
    CommException(std::string const& msg, const char* func, const char* file, int line)
        : Exception(std::string("communication error: ") + msg, func, file, line) {}
};

}  // namespace slate

#define slate_error(msg) throw ::slate::Exception(msg, __func__, __FILE__, __LINE__)

#define slate_error_if(cond) do { if (cond) \
    throw ::slate::Exception(std::string("error: ") + #cond, __func__, __FILE__, __LINE__); } while (0)

#define slate_error_if_msg(cond, msg) do { if (cond) \
    throw ::slate::Exception(std::string(msg), __func__, __FILE__, __LINE__); } while (0)

#define slate_assert(cond) do { if (!(cond)) \
    throw ::slate::Exception(std::string("assertion failed: ") + #cond, __func__, __FILE__, __LINE__); } while (0)

#define slate_not_implemented(msg) throw ::slate::NotImplemented(msg, __func__, __FILE__, __LINE__)
