// Core enumerations.  Semantics follow the reference's include/slate/enums.hh
// (Target :34-40, Option :63-99, NormScope :115, GridOrder :125, MOSI :138-143)
// and BLAS++/LAPACK++ enums (Op, Uplo, Diag, Side, Norm, Layout) which the
// reference takes from its blaspp submodule.
#pragma once

#include <cstdint>
#include <string>

namespace slate {

/// Location and method of computation (reference enums.hh:34-40).
/// On this framework HostTask/HostNest/HostBatch all run the C++/OpenMP host
/// kernels; Devices runs the gfx950 HIP kernels on this process's GPU.
enum class Target : char {
    Host      = 'H',
    HostTask  = 'T',
    HostNest  = 'N',
    HostBatch = 'B',
    Devices   = 'D',
};

inline bool is_host(Target t) { return t != Target::Devices; }

enum class Op     : char { NoTrans = 'N', Trans = 'T', ConjTrans = 'C' };
enum class Uplo   : char { Upper = 'U', Lower = 'L', General = 'G' };
enum class Diag   : char { NonUnit = 'N', Unit = 'U' };
enum class Side   : char { Left = 'L', Right = 'R' };
enum class Layout : char { ColMajor = 'C', RowMajor = 'R' };
enum class Norm   : char { One = '1', Two = '2', Inf = 'I', Fro = 'F', Max = 'M' };
enum class Job    : char { NoVec = 'N', Vec = 'V', AllVec = 'A', SomeVec = 'S', OverwriteVec = 'O' };
enum class Equed  : char { None = 'N', Row = 'R', Col = 'C', Both = 'B' };

/// Whether computing matrix norm, column norms, or row norms (enums.hh:115).
enum class NormScope : char { Columns = 'C', Rows = 'R', Matrix = 'M' };

/// Order to map processes to tile grid (enums.hh:125).
enum class GridOrder : char { Col = 'C', Row = 'R', Unknown = 'U' };

/// Layout conversion request (enums.hh:105).
enum class LayoutConvert : char { ColMajor = 'C', RowMajor = 'R', None = 'N' };

/// Eigenvalue method (enums.hh MethodEig).
enum class MethodEig : char { QR = 'Q', DC = 'D' };

/// Keys for options passed to routines (enums.hh:63-99).
enum class Option : char {
    ChunkSize,
    Lookahead,
    BlockSize,
    InnerBlocking,
    MaxPanelThreads,
    Tolerance,
    Target,
    HoldLocalWorkspace,
    Depth,
    MaxIterations,
    UseFallbackSolver,
    PivotThreshold,
    /// Mixed-precision solvers (gesv_mixed / posv_mixed): when classical
    /// refinement stalls or is projected to miss MaxIterations, continue with
    /// GMRES-IR preconditioned by the same low-precision factors before the
    /// full-precision fallback.  Not in the reference (default off: the
    /// reference semantics, classical refinement then fallback).
    EscalateGmres,

    PrintVerbose = 50,
    PrintEdgeItems,
    PrintWidth,
    PrintPrecision,

    MethodCholQR = 60,
    MethodEig,
    MethodGels,
    MethodGemm,
    MethodHemm,
    MethodLU,
    MethodTrsm,
};

const int HostNum    = -1;
const int AllDevices = -2;
const int AnyDevice  = -3;

/// Coherency state.  The reference keeps MOSI per tile instance
/// (enums.hh:138-143); here a matrix's local array has one host and one device
/// instance and the state is kept per instance at matrix granularity.
enum MOSI : short {
    Modified = 0x100,
    OnHold   = 0x1000,
    Shared   = 0x010,
    Invalid  = 0x001,
};
typedef short MOSI_State;

/// Kind of a tile buffer (reference Tile.hh:120-124).
enum class TileKind : char { Workspace = 'W', SlateOwned = 'S', UserOwned = 'U' };

//------------------------------------------------------------------------------
inline char to_char(Op v)     { return char(v); }
inline char to_char(Uplo v)   { return char(v); }
inline char to_char(Diag v)   { return char(v); }
inline char to_char(Side v)   { return char(v); }
inline char to_char(Norm v)   { return char(v); }
inline char to_char(Target v) { return char(v); }

inline Op    flip_trans(Op op, bool conj) { return op == Op::NoTrans ? (conj ? Op::ConjTrans : Op::Trans) : Op::NoTrans; }
inline Uplo  flip(Uplo u) { return u == Uplo::Lower ? Uplo::Upper : (u == Uplo::Upper ? Uplo::Lower : u); }
inline Side  flip(Side s) { return s == Side::Left ? Side::Right : Side::Left; }

const char* to_string(Target t);
const char* to_string(Op v);
const char* to_string(Uplo v);
const char* to_string(Norm v);
Target str2target(const std::string& s);
Norm   str2norm(const std::string& s);

}  // namespace slate
