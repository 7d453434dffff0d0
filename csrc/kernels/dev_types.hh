// Host/device-shared scalar types for the gfx950 kernels.  Compilable by a
// plain host C++ compiler (the launchers in kernels.hh use these types).
#pragma once

#include <cmath>
#include <cstdint>
#include <complex>
#include <cstring>

#if defined(__HIPCC__) || defined(__HIP__)
#define SLATE_HD __host__ __device__
#else
#define SLATE_HD
#endif

namespace slate_amd {
namespace dev {

//------------------------------------------------------------------------------
// POD complex type with the same layout as std::complex<R>.  Host code passes
// std::complex<R>* which is reinterpreted as cplx<R>* at the kernel boundary.
template <typename R>
struct alignas(2 * sizeof(R)) cplx {
    R re, im;
    SLATE_HD cplx() = default;
    SLATE_HD constexpr cplx(R r, R i = R(0)) : re(r), im(i) {}
};

template <typename T> struct real_type_t { using type = T; };
template <typename R> struct real_type_t<cplx<R>> { using type = R; };
template <typename T> using real_t = typename real_type_t<T>::type;

template <typename T> struct is_cplx { static constexpr bool value = false; };
template <typename R> struct is_cplx<cplx<R>> { static constexpr bool value = true; };

template <typename R> SLATE_HD inline cplx<R> operator+(cplx<R> a, cplx<R> b) { return {a.re + b.re, a.im + b.im}; }
template <typename R> SLATE_HD inline cplx<R> operator-(cplx<R> a, cplx<R> b) { return {a.re - b.re, a.im - b.im}; }
template <typename R> SLATE_HD inline cplx<R> operator-(cplx<R> a) { return {-a.re, -a.im}; }
template <typename R> SLATE_HD inline cplx<R> operator*(cplx<R> a, cplx<R> b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
template <typename R> SLATE_HD inline cplx<R> operator*(R a, cplx<R> b) { return {a * b.re, a * b.im}; }
template <typename R> SLATE_HD inline cplx<R> operator*(cplx<R> a, R b) { return {a.re * b, a.im * b}; }
template <typename R> SLATE_HD inline cplx<R>& operator+=(cplx<R>& a, cplx<R> b) { a.re += b.re; a.im += b.im; return a; }
template <typename R> SLATE_HD inline cplx<R>& operator-=(cplx<R>& a, cplx<R> b) { a.re -= b.re; a.im -= b.im; return a; }
template <typename R> SLATE_HD inline bool operator==(cplx<R> a, cplx<R> b) { return a.re == b.re && a.im == b.im; }
template <typename R> SLATE_HD inline bool operator!=(cplx<R> a, cplx<R> b) { return !(a == b); }
template <typename R> SLATE_HD inline cplx<R> operator/(cplx<R> a, cplx<R> b) {
    // Smith's algorithm (overflow-safe)
    if (fabs(b.re) >= fabs(b.im)) {
        R r = b.im / b.re, d = b.re + r * b.im;
        return {(a.re + a.im * r) / d, (a.im - a.re * r) / d};
    }
    R r = b.re / b.im, d = b.im + r * b.re;
    return {(a.re * r + a.im) / d, (a.im * r - a.re) / d};
}

SLATE_HD inline float  conj(float x)  { return x; }
SLATE_HD inline double conj(double x) { return x; }
template <typename R> SLATE_HD inline cplx<R> conj(cplx<R> x) { return {x.re, -x.im}; }

SLATE_HD inline float  real(float x)  { return x; }
SLATE_HD inline double real(double x) { return x; }
template <typename R> SLATE_HD inline R real(cplx<R> x) { return x.re; }
SLATE_HD inline float  imag(float)  { return 0; }
SLATE_HD inline double imag(double) { return 0; }
template <typename R> SLATE_HD inline R imag(cplx<R> x) { return x.im; }

/// host scalar type -> device scalar type
template <typename T> struct to_dev { using type = T; };
template <typename R> struct to_dev<std::complex<R>> { using type = cplx<R>; };
template <typename T> using dev_t = typename to_dev<T>::type;

template <typename T> inline dev_t<T>* dptr(T* p) { return reinterpret_cast<dev_t<T>*>(p); }
template <typename T> inline const dev_t<T>* dptr(const T* p) { return reinterpret_cast<const dev_t<T>*>(p); }
template <typename T> inline dev_t<T> dval(T v) { dev_t<T> r; static_assert(sizeof(r) == sizeof(v), ""); std::memcpy(&r, &v, sizeof(v)); return r; }

}  // namespace dev
}  // namespace slate_amd
