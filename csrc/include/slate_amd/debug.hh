// Debug utilities (reference src/auxiliary/Debug.hh:18-75, Debug.cc).
//
// The reference tracks one Tile per (i, j, device) with a MOSI state each, so
// its checks walk tile maps.  Here a process holds its whole local part in
// ONE ScaLAPACK-layout array per location (host, device), each with one MOSI
// state, so the same questions are asked of those instances:
//   * checkTilesLives   - every local tile is backed by a live, valid instance
//   * checkTilesLayout  - column-major local arrays with ld >= local rows
//   * printTiles        - per-tile map: owner, host/device MOSI state
//   * diffLapackMatrices- tile map of where two column-major matrices differ
//   * memory            - the caching device allocator's blocks and bytes
//                         (checkDeviceMemoryLeaks: bytes still in use)
// Everything is a no-op unless Debug::on() (or SLATE_DEBUG=1) except the
// explicit report/print calls, which always run.
#pragma once

#include "matrix.hh"

#include <cstdint>
#include <string>

namespace slate {

class Debug {
public:
    static void on();
    static void off();
    static bool enabled();

    /// Tile map of where A and B (m x n, column-major) differ by more than
    /// tol * max|A|: '.' equal tile, '#' differing tile.  Returns the number
    /// of differing tiles; the map goes to `out` (and stdout when enabled).
    template <typename T>
    static int64_t diffLapackMatrices(int64_t m, int64_t n, T const* A, int64_t lda, T const* B, int64_t ldb,
                                      int64_t mb, int64_t nb, double tol = 0.0, std::string* out = nullptr);

    /// Number of local tiles that are not backed by a live valid instance
    /// (no host or device array, or every instance Invalid).
    template <typename T>
    static int64_t checkTilesLives(BaseMatrix<T> const& A);

    /// true if every local instance is column-major with ld >= local rows
    template <typename T>
    static bool checkTilesLayout(BaseMatrix<T> const& A);

    /// Per-tile map of this process's view: for each tile the owner rank,
    /// and for local tiles the host/device MOSI letters (M, O, S, I, '-' =
    /// no instance).  Returned as text (and printed when enabled).
    template <typename T>
    static std::string printTiles(BaseMatrix<T> const& A);

    /// Device allocator report: blocks / bytes in use and cached.
    static std::string printNumFreeMemBlocks();
    /// Bytes of device memory still handed out by the allocator.
    static size_t checkDeviceMemoryLeaks();
    /// Bytes of pinned host memory still handed out.
    static size_t checkHostMemoryLeaks();
};

}  // namespace slate
