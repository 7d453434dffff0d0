// Algorithm selection (reference include/slate/method.hh:25-315).
#pragma once

#include "types.hh"

#include <algorithm>
#include <string>

namespace slate {

typedef int Method;
const Method baseMethodError = -1;
const Method baseMethodAuto = 0;

namespace MethodTrsm {
const Method Error = baseMethodError, Auto = baseMethodAuto, TrsmA = 1, TrsmB = 2;
inline Method str2method(std::string s) {
    std::transform(s.begin(), s.end(), s.begin(), ::tolower);
    if (s == "auto") return Auto;
    if (s == "a" || s == "trsma") return TrsmA;
    if (s == "b" || s == "trsmb") return TrsmB;
    throw Exception("unknown trsm method");
}
}  // namespace MethodTrsm

namespace MethodGemm {
const Method Error = baseMethodError, Auto = baseMethodAuto, GemmA = 1, GemmC = 2;
/// GemmA (stationary A, reduce C) when B is a single block column, else
/// GemmC (SUMMA, stationary C); reference method.hh:87-98.
template <typename M>
inline Method select_algo(M const& A, M const& B, Options const&) {
    (void)A;
    return B.nt() < 2 ? GemmA : GemmC;
}
inline Method str2method(std::string s) {
    std::transform(s.begin(), s.end(), s.begin(), ::tolower);
    if (s == "auto") return Auto;
    if (s == "a" || s == "gemma") return GemmA;
    if (s == "c" || s == "gemmc") return GemmC;
    throw Exception("unknown gemm method");
}
}  // namespace MethodGemm

namespace MethodHemm {
const Method Error = baseMethodError, Auto = baseMethodAuto, HemmA = 1, HemmC = 2;
inline Method str2method(std::string s) {
    std::transform(s.begin(), s.end(), s.begin(), ::tolower);
    if (s == "auto") return Auto;
    if (s == "a" || s == "hemma") return HemmA;
    if (s == "c" || s == "hemmc") return HemmC;
    throw Exception("unknown hemm method");
}
}  // namespace MethodHemm

/// How cholqr forms A^H A (reference method.hh:181-232): HerkC (triangle
/// only, default on devices), GemmA / GemmC (full product by the stationary-A
/// or SUMMA gemm; GemmA is the host default).
namespace MethodCholQR {
const Method Error = baseMethodError, Auto = baseMethodAuto, HerkC = 1, GemmA = 2, GemmC = 3;
inline Method select_algo(Target target) { return target == Target::Devices ? HerkC : GemmA; }
inline Method str2method(std::string s) {
    std::transform(s.begin(), s.end(), s.begin(), ::tolower);
    if (s == "auto") return Auto;
    if (s == "herkc" || s == "herk") return HerkC;
    if (s == "gemma") return GemmA;
    if (s == "gemmc" || s == "gemm") return GemmC;
    throw Exception("unknown cholQR method");
}
inline const char* method2str(Method m) {
    switch (m) {
        case Auto: return "auto";
        case HerkC: return "herkC";
        case GemmA: return "gemmA";
        case GemmC: return "gemmC";
        default: return "error";
    }
}
}  // namespace MethodCholQR

namespace MethodGels {
const Method Error = baseMethodError, Auto = baseMethodAuto, Geqrf = 1, Cholqr = 2;
inline Method str2method(std::string s) {
    std::transform(s.begin(), s.end(), s.begin(), ::tolower);
    if (s == "auto") return Auto;
    if (s == "qr" || s == "geqrf") return Geqrf;
    if (s == "cholqr") return Cholqr;
    throw Exception("unknown gels method");
}
}  // namespace MethodGels

namespace MethodLU {
const Method Error = baseMethodError, Auto = baseMethodAuto, PartialPiv = 1, CALU = 2, NoPiv = 3;
inline Method str2method(std::string s) {
    std::transform(s.begin(), s.end(), s.begin(), ::tolower);
    if (s == "auto" || s == "ppiv" || s == "partialpiv") return PartialPiv;
    if (s == "calu" || s == "tntpiv") return CALU;
    if (s == "nopiv") return NoPiv;
    throw Exception("unknown LU method");
}
}  // namespace MethodLU

}  // namespace slate
