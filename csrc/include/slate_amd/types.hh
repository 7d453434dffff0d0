// Options, pivots and scalar traits (reference include/slate/types.hh:32-251).
#pragma once

#include "enums.hh"
#include "exception.hh"

#include <complex>
#include <map>
#include <vector>
#include <limits>
#include <type_traits>
#include <cmath>

namespace slate {

//------------------------------------------------------------------------------
// scalar traits
template <typename T> struct real_type_traits { using type = T; };
template <typename R> struct real_type_traits<std::complex<R>> { using type = R; };
template <typename T> using real_type = typename real_type_traits<T>::type;

template <typename T> struct is_complex : std::false_type {};
template <typename R> struct is_complex<std::complex<R>> : std::true_type {};
template <typename T> constexpr bool is_complex_v = is_complex<T>::value;

template <typename T> inline T conj(T x) { return x; }
template <typename R> inline std::complex<R> conj(std::complex<R> x) { return std::conj(x); }
template <typename T> inline real_type<T> real(T x) { return std::real(x); }
template <typename T> inline real_type<T> imag(T x) { return std::imag(x); }
/// |re| + |im|
template <typename T> inline real_type<T> cabs1(T x) { return std::abs(std::real(x)) + std::abs(std::imag(x)); }

/// scalar type code (for comm, dispatch, bindings)
enum class ScalarType : char { Int32 = 'i', Int64 = 'l', Float32 = 's', Float64 = 'd', Complex64 = 'c', Complex128 = 'z', Byte = 'b' };
template <typename T> constexpr ScalarType scalar_type();
template <> constexpr ScalarType scalar_type<float>()                { return ScalarType::Float32; }
template <> constexpr ScalarType scalar_type<double>()               { return ScalarType::Float64; }
template <> constexpr ScalarType scalar_type<std::complex<float>>()  { return ScalarType::Complex64; }
template <> constexpr ScalarType scalar_type<std::complex<double>>() { return ScalarType::Complex128; }
template <> constexpr ScalarType scalar_type<int>()                  { return ScalarType::Int32; }
template <> constexpr ScalarType scalar_type<int64_t>()              { return ScalarType::Int64; }

//------------------------------------------------------------------------------
/// Value of an option (reference types.hh:32).
class OptionValue {
public:
    OptionValue() : i_(0), d_(0) {}
    OptionValue(int i) : i_(i), d_(i) {}
    OptionValue(int64_t i) : i_(i), d_(double(i)) {}
    OptionValue(double d) : i_(int64_t(d)), d_(d) {}
    OptionValue(bool b) : i_(b), d_(b) {}
    OptionValue(Target t) : i_(int64_t(t)), d_(0) {}
    OptionValue(MethodEig m) : i_(int64_t(m)), d_(0) {}
    int64_t i_;
    double d_;
};

using Options = std::map<Option, OptionValue>;

/// get_option (reference types.hh:193-218)
template <typename T>
inline T get_option(Options const& opts, Option key, T defval) {
    auto it = opts.find(key);
    if (it == opts.end()) return defval;
    if constexpr (std::is_same_v<T, double> || std::is_same_v<T, float>)
        return T(it->second.d_);
    else
        return T(it->second.i_);
}

/// Target used when the options name none: the caller's default, unless the
/// thread runs a driver on the parts of multi-device matrices (spread.hh),
/// whose data lives on the devices -- then Target::Devices.
inline Target& thread_default_target() { thread_local Target t = Target(0); return t; }
inline Target get_target(Options const& opts, Target def = Target::HostTask) {
    auto it = opts.find(Option::Target);
    if (it != opts.end()) return Target(char(it->second.i_));
    return thread_default_target() != Target(0) ? thread_default_target() : def;
}

//------------------------------------------------------------------------------
/// Pivot: tile index + element offset within the tile (reference types.hh:65).
class Pivot {
public:
    Pivot() : tile_index_(0), element_offset_(0) {}
    Pivot(int64_t tile_index, int64_t element_offset)
        : tile_index_(tile_index), element_offset_(element_offset) {}
    int64_t tileIndex() const { return tile_index_; }
    int64_t elementOffset() const { return element_offset_; }
    bool operator==(Pivot const& o) const { return tile_index_ == o.tile_index_ && element_offset_ == o.element_offset_; }
private:
    int64_t tile_index_, element_offset_;
};

/// One vector of pivots per block column (reference types.hh:98).
/// Pivot k*nb + t of block k is stored in pivots[k][t] as the (tile, offset)
/// of the row (relative to the diagonal block row k) it was swapped with.
using Pivots = std::vector<std::vector<Pivot>>;

}  // namespace slate
