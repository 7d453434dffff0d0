// Distributed tiled matrices.
//
// Reference: BaseMatrix.hh (view fields :766-800, MOSI tileGet :2640-2723),
// MatrixStorage.hh (TileNode map :35-160, 2D block-cyclic default :478-516),
// Matrix.hh (fromLAPACK :293, fromScaLAPACK :347, fromDevices :397,
// emptyLike :432, insertLocalTiles :832), and the Trapezoid/Triangular/
// Symmetric/Hermitian/Band subclasses.
//
// MI355X-first storage: instead of a std::map of separately allocated nb x nb
// tiles, every process holds ONE contiguous column-major local array (the
// ScaLAPACK local layout of the 2D block-cyclic distribution) on its GPU
// and/or host.  A tile is a view into it.  Because local indices are monotone
// in global indices, the local part of ANY sub-matrix view is a contiguous
// strided block, so a trailing update is one large local GEMM per process.
// Coherency between the host and device instance is MOSI at matrix
// granularity (MatrixStorage::get).
#pragma once

#include "types.hh"
#include "util.hh"
#include "grid.hh"
#include "device.hh"

#include <functional>
#include <map>
#include <set>
#include <memory>
#include <tuple>

namespace slate {

class InprocGroup;   // inproc.hh

//------------------------------------------------------------------------------
/// Non-owning view of one tile (reference Tile.hh:395-419).
template <typename T>
struct Tile {
    T* data = nullptr;
    int64_t mb = 0, nb = 0, stride = 0;
    Op op = Op::NoTrans;
    Uplo uplo = Uplo::General;
    int device = HostNum;
    /// memory layout of the stored mb x nb block: ColMajor (element (r, c)
    /// at data[r + c stride]) or RowMajor (at data[c + r stride]); see
    /// BaseMatrix::tileLayoutConvert
    Layout layout = Layout::ColMajor;
    int64_t mb_() const { return op == Op::NoTrans ? mb : nb; }
    int64_t nb_() const { return op == Op::NoTrans ? nb : mb; }
    /// element (i, j) of the (op-applied) tile, host tiles only
    T at(int64_t i, int64_t j) const {
        const int64_t r = op == Op::NoTrans ? i : j, c = op == Op::NoTrans ? j : i;
        T v = layout == Layout::ColMajor ? data[r + c * stride] : data[c + r * stride];
        return op == Op::ConjTrans ? slate::conj(v) : v;
    }
};

/// Local strided block (storage orientation).
template <typename T>
struct LocalBlock {
    T* ptr = nullptr;
    int64_t m = 0, n = 0, ld = 1;
    bool empty() const { return m <= 0 || n <= 0; }
    T* at(int64_t i, int64_t j) const { return ptr + i + j * ld; }
};

/// Largest single local-array allocation (bytes) of any matrix since the last
/// reset -- lets tests assert that a driver made no n x n temporary.
size_t storage_alloc_max();
void storage_alloc_reset();

//------------------------------------------------------------------------------
/// Per-process storage of a distributed matrix.
template <typename T>
class MatrixStorage {
public:
    /// rsrc/csrc: process row/column owning the first tile row/column
    /// (ScaLAPACK descriptor RSRC/CSRC).
    MatrixStorage(int64_t m, int64_t n, int64_t mb, int64_t nb, GridPtr grid, int rsrc = 0, int csrc = 0);

    /// Arbitrary distribution (reference Matrix.hh:207-212 lambda constructor):
    /// tile row/column sizes and the owning world rank of every tile.  The
    /// tiles a process owns are packed column-major one after another (ld =
    /// tile rows) in one host / device buffer.
    struct Layout {
        int64_t mt = 0, nt = 0;
        std::vector<int64_t> rs, cs;       // tile row / column starts (mt + 1, nt + 1)
        std::vector<int> owner;            // world rank of tile (i, j) at i + j mt
        std::vector<int64_t> toff;         // my tiles: element offset in the local buffer, else -1
    };
    MatrixStorage(int64_t m, int64_t n, std::function<int64_t(int64_t)> const& tile_mb,
                  std::function<int64_t(int64_t)> const& tile_nb,
                  std::function<int(int64_t, int64_t)> const& tile_rank, GridPtr grid);
    std::shared_ptr<Layout> layout;
    bool general() const { return layout != nullptr; }

    /// Band-only storage (reference BaseBandMatrix.hh:219-258: only the tiles
    /// that intersect the band exist).  Tile (i, j) is stored iff
    /// j - band_ut <= i <= j + band_lt (tile bandwidths).  Within each local
    /// tile column the stored tiles are a contiguous range of local rows
    /// [boff, bend); the allocation is lld (= the largest range, padded) x
    /// nloc, element (lr, lc) at (lr - boff[lc / nb]) + lc * lld.  O(n x
    /// bandwidth) memory instead of the dense local array.
    struct BandTag {};
    MatrixStorage(int64_t m, int64_t n, int64_t nb, GridPtr grid, int64_t kl, int64_t ku, BandTag);
    bool banded = false;
    int64_t band_lt = 0, band_ut = 0;
    std::vector<int64_t> boff, bend;   // per local tile column
    /// host/device pointer of local element (lr, lc), or null when the tile
    /// is outside the stored band (banded storage) -- dense storage: always
    T* local_ptr(Loc loc, int64_t lr, int64_t lc) const {
        T* base = raw(loc);
        if (!base) return nullptr;
        const int64_t ld = this->ld(loc);
        if (!banded) return base + lr + lc * ld;
        const int64_t lj = lc / nb;
        if (lr < boff[lj] || lr >= bend[lj]) return nullptr;
        return base + (lr - boff[lj]) + lc * ld;
    }
    ~MatrixStorage();
    /// Remote tiles received with tileRecv / tileBcast (reference workspace
    /// tiles, MatrixStorage.hh tileInsertWorkspace): contiguous mb x nb
    /// buffers at `loc`, keyed by absolute storage tile (row, col).  Local
    /// tiles whose layout was converted to RowMajor are listed in
    /// tile_layouts.
    struct WsTile { T* ptr = nullptr; int64_t mb = 0, nb = 0; Loc loc = Loc::Host; };
    std::map<std::pair<int64_t, int64_t>, WsTile> ws_tiles;
    std::map<std::pair<int64_t, int64_t>, slate::Layout> tile_layouts;
    /// workspace tile (si, sj) of mb x nb at loc, allocated if missing
    T* ws_tile(int64_t si, int64_t sj, int64_t mb, int64_t nb, Loc loc);
    void ws_erase(int64_t si, int64_t sj);
    MatrixStorage(MatrixStorage const&) = delete;
    MatrixStorage& operator=(MatrixStorage const&) = delete;

    /// Multi-device storage (reference: one MPI rank spreads its tiles over
    /// all of its GPUs, tileDevice = func::device_1d_grid, MatrixStorage.hh:
    /// 503-506; Matrix::fromDevices(Aarray, num_devices), Matrix.hh:396-404).
    /// The matrix lives on the ranks of an in-process group (inproc.hh):
    /// parts[r] is rank r's block-cyclic local storage on group->grid(r), on
    /// rank r's device.  This caller-side storage holds no data; drivers
    /// called with it run on the group's ranks directly on the parts
    /// (spread.hh) -- no scatter or gather per call.
    std::shared_ptr<InprocGroup> group;
    std::vector<std::shared_ptr<MatrixStorage<T>>> parts;
    bool multi() const { return !parts.empty(); }

    int64_t m, n, mb, nb;
    GridPtr grid;
    int rsrc, csrc;
    int64_t mloc, nloc, lld;
    /// my process row/column relative to the source (for numroc)
    int rrel() const { return (grid->myrow() - rsrc + grid->p()) % grid->p(); }
    int crel() const { return (grid->mycol() - csrc + grid->q()) % grid->q(); }
    int row_owner(int64_t tile_row) const { return int((tile_row + rsrc) % grid->p()); }
    int col_owner(int64_t tile_col) const { return int((tile_col + csrc) % grid->q()); }

    /// Attach user memory as the origin instance (reference TileKind::UserOwned).
    void attach(T* ptr, int64_t ld, Loc loc);
    /// Allocate the instance at `loc` if missing (SlateOwned), no data movement.
    void allocate(Loc loc);
    bool has(Loc loc) const { return (loc == Loc::Host ? host_ : dev_) != nullptr; }

    /// Coherent access (MOSI at matrix granularity): makes the instance at
    /// `loc` valid (copying from the other one if needed) and, when
    /// `for_write`, invalidates the other instance.  Returns the base pointer.
    T* get(Loc loc, bool for_write);
    /// Pointer without coherency action.
    T* raw(Loc loc) const { return loc == Loc::Host ? host_ : dev_; }
    int64_t ld(Loc loc) const { return loc == Loc::Host ? host_ld_ : dev_ld_; }
    MOSI_State state(Loc loc) const { return loc == Loc::Host ? host_state_ : dev_state_; }
    /// Mark the instance at loc modified (others invalid).
    void modified(Loc loc);
    /// Copy the modified instance back to the origin (tileUpdateAllOrigin).
    void update_origin();
    Loc origin() const { return origin_; }
    /// Free the non-origin instance (releaseLocalWorkspace analog).
    void release_workspace();
    TileKind kind() const { return kind_; }

private:
    void copy_instance(Loc to);
    T* host_ = nullptr;
    T* dev_ = nullptr;
    int64_t host_ld_ = 0, dev_ld_ = 0;
    bool host_owned_ = false, dev_owned_ = false;
    MOSI_State host_state_ = Invalid, dev_state_ = Invalid;
    Loc origin_ = Loc::Host;
    TileKind kind_ = TileKind::SlateOwned;
};

/// Matrix kind tag (for the derived view classes).
enum class MatrixKind : char {
    General = 'G', Trapezoid = 'Z', Triangular = 'T', Symmetric = 'S', Hermitian = 'H',
    Band = 'B', TriangularBand = 't', HermitianBand = 'h',
};

//------------------------------------------------------------------------------
/// A view of a distributed matrix (reference BaseMatrix.hh).  Offsets r0/c0
/// and dims m_/n_ are in storage orientation; op() maps logical (i, j) to
/// storage (j, i) when transposed.
template <typename T>
class BaseMatrix {
public:
    using value_type = T;
    BaseMatrix() = default;
    BaseMatrix(std::shared_ptr<MatrixStorage<T>> s)
        : storage_(s), r0_(0), c0_(0), m_(s->m), n_(s->n) {}

    // ---- dimensions (op applied)
    int64_t m() const { return op_ == Op::NoTrans ? m_ : n_; }
    int64_t n() const { return op_ == Op::NoTrans ? n_ : m_; }
    int64_t mt() const { return op_ == Op::NoTrans ? smt() : snt(); }
    int64_t nt() const { return op_ == Op::NoTrans ? snt() : smt(); }
    int64_t tileMb(int64_t i) const { return op_ == Op::NoTrans ? srow_size(i) : scol_size(i); }
    int64_t tileNb(int64_t j) const { return op_ == Op::NoTrans ? scol_size(j) : srow_size(j); }
    Op op() const { return op_; }
    Uplo uplo() const { return uplo_; }
    /// uplo as seen in storage orientation
    Uplo uplo_physical() const { return op_ == Op::NoTrans ? uplo_ : flip(uplo_); }
    Diag diag() const { return diag_; }
    MatrixKind matrix_kind() const { return kind_; }

    // ---- distribution
    GridPtr grid() const { return storage_->grid; }
    int mpiRank() const { return storage_->grid->rank(); }
    int64_t mb() const { return storage_->mb; }
    int64_t nb() const { return storage_->nb; }
    /// rank owning logical tile (i, j)
    int tileRank(int64_t i, int64_t j) const {
        int64_t si, sj; to_storage(i, j, si, sj);
        if (storage_->general()) return storage_->layout->owner[si + sj * storage_->layout->mt];
        auto& g = *storage_->grid;
        return g.rank_of(storage_->row_owner(stile_r(si)), storage_->col_owner(stile_c(sj)));
    }
    /// arbitrary (lambda) distribution: drivers work on a block-cyclic copy
    bool arbitrary_layout() const { return storage_ && storage_->general(); }
    bool tileIsLocal(int64_t i, int64_t j) const { return tileRank(i, j) == mpiRank(); }
    int tileDevice(int64_t i, int64_t j) const { return tileIsLocal(i, j) ? 0 : HostNum; }
    /// process row / column owning storage tile-row/col (storage orientation)
    int srow_owner(int64_t si) const { return storage_->row_owner(stile_r(si)); }
    int scol_owner(int64_t sj) const { return storage_->col_owner(stile_c(sj)); }
    void gridinfo(GridOrder& order, int& p, int& q, int& myrow, int& mycol) const {
        auto& g = *storage_->grid;
        order = g.order(); p = g.p(); q = g.q(); myrow = g.myrow(); mycol = g.mycol();
    }
    int num_devices() const { return device::available() ? 1 : 0; }

    // ---- views (tile index ranges are inclusive, as in the reference)
    /// sub-matrix of logical tiles [i1..i2] x [j1..j2]
    BaseMatrix sub(int64_t i1, int64_t i2, int64_t j1, int64_t j2) const;
    /// element slice rows [r1..r2], cols [c1..c2] (inclusive)
    BaseMatrix slice(int64_t r1, int64_t r2, int64_t c1, int64_t c2) const;

    /// storage-orientation element offsets/dims
    int64_t row0() const { return r0_; }
    int64_t col0() const { return c0_; }
    int64_t srows() const { return m_; }
    int64_t scols() const { return n_; }

    // ---- local data access
    /// Local strided block of this view at `loc` (storage orientation).
    /// Applies coherency: for_write invalidates the other instance.
    LocalBlock<T> local(Loc loc, bool for_write = false) const;
    /// Local block without coherency action (storage must be valid at loc).
    LocalBlock<T> local_raw(Loc loc) const;
    /// Local rows/cols ranges in the local array (storage orientation)
    int64_t lrow_begin() const;
    int64_t lrow_end() const;
    int64_t lcol_begin() const;
    int64_t lcol_end() const;
    /// View of logical tile (i, j): a local tile, or a remote one received
    /// into workspace by tileRecv / tileBcast.
    Tile<T> tile(int64_t i, int64_t j, Loc loc) const;

    // ---- tile-level communication and layout (reference BaseMatrix.hh
    // tileSend / tileRecv / tileBcast / tileBcastToSet / tileLayoutConvert,
    // Tile.hh send / recv / bcast / layoutConvert).  Messages go over the
    // grid's world communicator (RCCL on the device, the native TCP mesh or
    // the in-process transport on the host); a strided tile is packed into one
    // contiguous message.  Point-to-point order is per peer, so `tag` is
    // accepted for source compatibility and not needed.
    /// local tile, or a received workspace tile
    bool tileExists(int64_t i, int64_t j) const;
    Layout tileLayout(int64_t i, int64_t j) const;
    /// send tile (i, j) (local) to dst_rank, which calls tileRecv
    void tileSend(int64_t i, int64_t j, int dst_rank, int tag = 0) const;
    /// receive tile (i, j) from src_rank: in place when local, else into a
    /// workspace tile; `layout` is the layout the tile is left in
    void tileRecv(int64_t i, int64_t j, int src_rank, Layout layout = Layout::ColMajor, int tag = 0);
    /// broadcast tile (i, j) from its owner to every rank owning a tile of B
    /// (called by every rank of the grid; others return at once)
    void tileBcast(int64_t i, int64_t j, BaseMatrix<T> const& B, Layout layout = Layout::ColMajor, int tag = 0);
    /// broadcast to an explicit rank set (binomial tree rooted at the owner);
    /// every rank of the set (and the owner) calls it
    void tileBcastToSet(int64_t i, int64_t j, std::set<int> const& ranks, Layout layout = Layout::ColMajor);
    /// convert tile (i, j) in place between column- and row-major: square
    /// tiles anywhere, rectangular ones only as contiguous workspace tiles
    void tileLayoutConvert(int64_t i, int64_t j, Layout layout);
    /// drop a received workspace tile (local tiles are kept)
    void tileErase(int64_t i, int64_t j);
    Tile<T> operator()(int64_t i, int64_t j) const { return tile(i, j, Loc::Host); }

    /// Element access (global logical indices), host instance, local only.
    T& elem(int64_t i, int64_t j);

    std::shared_ptr<MatrixStorage<T>> storage() const { return storage_; }
    /// multi-device matrix: spread over the devices of an in-process group
    bool is_multi_device() const { return storage_ && storage_->multi(); }
    /// the view v (of another storage with the same geometry) on this storage
    BaseMatrix rebase(BaseMatrix const& v) const {
        BaseMatrix r = v;
        r.storage_ = storage_;
        return r;
    }
    /// the same view (offsets, op, uplo, diag, kind, bands) on in-process
    /// rank r's part of a multi-device matrix
    BaseMatrix on_part(int r) const {
        slate_error_if_msg(!is_multi_device(), "on_part: not a multi-device matrix");
        BaseMatrix v = *this;
        v.storage_ = storage_->parts.at(size_t(r));
        return v;
    }
    bool aligned() const { return r0_ % storage_->mb == 0 && c0_ % storage_->nb == 0; }

    /// Make the host or device instance valid; mark modified.
    void tileGetAllForReading(Loc loc) const { storage_->get(loc, false); }
    void tileGetAllForWriting(Loc loc) const { storage_->get(loc, true); }
    void tileUpdateAllOrigin() const { storage_->update_origin(); }
    void releaseWorkspace() const { storage_->release_workspace(); }

    // ---- op flips (friends transpose/conj_transpose)
    BaseMatrix transpose_view(bool conj) const {
        BaseMatrix r = *this;
        r.uplo_ = flip(uplo_);
        std::swap(r.kl_, r.ku_);
        if (op_ == Op::NoTrans) r.op_ = conj ? Op::ConjTrans : Op::Trans;
        else {
            slate_error_if_msg((op_ == Op::ConjTrans) != conj && is_complex_v<T>,
                               "cannot mix transpose and conj_transpose");
            r.op_ = Op::NoTrans;
        }
        return r;
    }

    // mutable meta (used by derived-class constructors)
    void set_uplo(Uplo u) { uplo_ = u; }
    void set_diag(Diag d) { diag_ = d; }
    void set_kind(MatrixKind k) { kind_ = k; }
    int64_t kl() const { return kl_; }
    int64_t ku() const { return ku_; }
    void set_band(int64_t kl, int64_t ku) { kl_ = kl; ku_ = ku; }

    /// (drop every local tile back to column-major: drivers read local
    /// arrays as column-major)
    void tileLayoutReset();

protected:
    void to_storage(int64_t i, int64_t j, int64_t& si, int64_t& sj) const {
        if (op_ == Op::NoTrans) { si = i; sj = j; } else { si = j; sj = i; }
    }
    /// absolute storage tile of view storage tile (si, sj): workspace key
    std::pair<int64_t, int64_t> skey(int64_t si, int64_t sj) const {
        return storage_->general() ? std::make_pair(si, sj) : std::make_pair(stile_r(si), stile_c(sj));
    }
    // storage-orientation tile counts and sizes of this view
    int64_t stile_r0() const { return r0_ / storage_->mb; }
    int64_t stile_c0() const { return c0_ / storage_->nb; }
    int64_t stile_r(int64_t si) const { return stile_r0() + si; }
    int64_t stile_c(int64_t sj) const { return stile_c0() + sj; }
    int64_t smt() const {
        if (storage_->general()) return storage_->layout->mt;
        return m_ == 0 ? 0 : (r0_ + m_ - 1) / storage_->mb - stile_r0() + 1;
    }
    int64_t snt() const {
        if (storage_->general()) return storage_->layout->nt;
        return n_ == 0 ? 0 : (c0_ + n_ - 1) / storage_->nb - stile_c0() + 1;
    }
    int64_t srow_start(int64_t si) const {
        if (storage_->general()) return storage_->layout->rs[si];
        return std::max(r0_, stile_r(si) * storage_->mb);
    }
    int64_t scol_start(int64_t sj) const {
        if (storage_->general()) return storage_->layout->cs[sj];
        return std::max(c0_, stile_c(sj) * storage_->nb);
    }
    int64_t srow_size(int64_t si) const {
        if (storage_->general()) return storage_->layout->rs[si + 1] - storage_->layout->rs[si];
        return std::min(r0_ + m_, (stile_r(si) + 1) * storage_->mb) - srow_start(si);
    }
    int64_t scol_size(int64_t sj) const {
        if (storage_->general()) return storage_->layout->cs[sj + 1] - storage_->layout->cs[sj];
        return std::min(c0_ + n_, (stile_c(sj) + 1) * storage_->nb) - scol_start(sj);
    }

    std::shared_ptr<MatrixStorage<T>> storage_;
    int64_t r0_ = 0, c0_ = 0, m_ = 0, n_ = 0;
    Op op_ = Op::NoTrans;
    Uplo uplo_ = Uplo::General;
    Diag diag_ = Diag::NonUnit;
    MatrixKind kind_ = MatrixKind::General;
    int64_t kl_ = 0, ku_ = 0;
};

//------------------------------------------------------------------------------
// Concrete matrix classes.  They share BaseMatrix's storage/views and differ
// in the meta-data (kind, uplo, diag, bandwidths) that drivers dispatch on.

template <typename T> class Matrix;

template <typename T>
class Matrix : public BaseMatrix<T> {
public:
    using BaseMatrix<T>::BaseMatrix;
    Matrix() = default;
    /// Distributed m x n matrix with nb x nb tiles on a p x q grid (storage
    /// allocated lazily by insertLocalTiles), reference Matrix.hh:41-55.
    Matrix(int64_t m, int64_t n, int64_t nb, GridPtr grid = nullptr)
        : Matrix(m, n, nb, nb, grid) {}
    Matrix(int64_t m, int64_t n, int64_t mb, int64_t nb, GridPtr grid, int rsrc = 0, int csrc = 0)
        : BaseMatrix<T>(std::make_shared<MatrixStorage<T>>(m, n, mb, nb, grid ? grid : default_grid(), rsrc, csrc)) {}
    explicit Matrix(BaseMatrix<T> const& b) : BaseMatrix<T>(b) { this->set_kind(MatrixKind::General); }
    /// Band-only storage for an m x n matrix of bandwidths kl / ku (see
    /// MatrixStorage::BandTag); used by the sized band-matrix constructors.
    static Matrix banded(int64_t m, int64_t n, int64_t kl, int64_t ku, int64_t nb, GridPtr grid) {
        return Matrix(BaseMatrix<T>(std::make_shared<MatrixStorage<T>>(
            m, n, nb, grid ? grid : default_grid(), kl, ku, typename MatrixStorage<T>::BandTag{})));
    }
    /// Arbitrary distribution with non-uniform tiles (reference Matrix.hh:
    /// 207-212): tileMb(i), tileNb(j), tileRank({i, j}) (world rank),
    /// tileDevice (one GPU per process here, accepted for API parity).  The
    /// grid supplies the communicators; drivers run on a block-cyclic copy.
    Matrix(int64_t m, int64_t n, std::function<int64_t(int64_t)> tileMb, std::function<int64_t(int64_t)> tileNb,
           std::function<int(std::tuple<int64_t, int64_t>)> tileRank,
           std::function<int(std::tuple<int64_t, int64_t>)> tileDevice, GridPtr grid = nullptr)
        : BaseMatrix<T>(std::make_shared<MatrixStorage<T>>(
              m, n, tileMb, tileNb,
              [tileRank](int64_t i, int64_t j) { return tileRank(std::make_tuple(i, j)); },
              grid ? grid : default_grid())) { (void)tileDevice; }

    /// Wrap a column-major LAPACK array (1 x 1 grid or replicated-rank use).
    static Matrix fromLAPACK(int64_t m, int64_t n, T* A, int64_t lda, int64_t nb, Loc loc = Loc::Host);
    /// Wrap a ScaLAPACK local array (2D block-cyclic on `grid`).
    static Matrix fromScaLAPACK(int64_t m, int64_t n, T* A, int64_t lld, int64_t mb, int64_t nb,
                                GridPtr grid, Loc loc = Loc::Host, int rsrc = 0, int csrc = 0);
    /// Wrap a device-resident local array (one GPU per process).
    static Matrix fromDevices(int64_t m, int64_t n, T* dA, int64_t lld, int64_t mb, int64_t nb, GridPtr grid) {
        return fromScaLAPACK(m, n, dA, lld, mb, nb, grid, Loc::Device);
    }
    /// Reference fromDevices (Matrix.hh:396-404, 529-563): one process, its
    /// tiles 1-D block-cyclic over num_devices GPUs by tile column (tile
    /// column j on device j % num_devices); Aarray[d] is device d's local
    /// array (its tile columns side by side, leading dimension lda).  The
    /// matrix is a multi-device matrix over a 1 x num_devices in-process
    /// group on devices 0 .. num_devices-1.  p x q must be 1 x 1 (a
    /// multi-process job runs one GPU per process: use the overload above).
    /// Without a GPU (CPU builds and tests) the arrays are host memory.
    static Matrix fromDevices(int64_t m, int64_t n, T** Aarray, int num_devices, int64_t lda, int64_t mb,
                              int64_t nb, int p = 1, int q = 1);
    /// New multi-device matrix, 2-D block-cyclic over the near-square grid
    /// of num_devices in-process ranks (0: every GPU the process may use;
    /// 8 GPUs -> 2 x 4), allocated on the devices.  Every driver that accepts
    /// it (gemm, trsm, herk, getrf / getrs / gesv, potrf / potrs / posv,
    /// geqrf / gels, the mixed-precision solvers, heev, svd, norm, copy,
    /// add, scale, set) runs on those ranks in place.
    static Matrix multiDevice(int64_t m, int64_t n, int64_t mb, int64_t nb, int num_devices = 0);
    /// Caller-side multi-device matrix over `group` whose parts are the
    /// per-rank matrices parts[r] (made on the group's rank threads, same
    /// geometry, whole views): drivers' distributed outputs (QR T factors).
    static Matrix fromParts(std::shared_ptr<InprocGroup> const& group, std::vector<Matrix<T>> const& parts);
    /// Gather the whole matrix into a column-major host array (every rank
    /// of a multi-process grid, or the caller of a multi-device matrix).
    void gather(T* A, int64_t lda) const;

    /// Allocate local storage at the target's location (Matrix.hh:832).
    void insertLocalTiles(Target target = Target::Host) const {
        if (this->storage_->multi()) { insert_parts(target); return; }
        auto loc = target == Target::Devices ? Loc::Device : Loc::Host;
        auto other = loc == Loc::Device ? Loc::Host : Loc::Device;
        bool fresh = !(this->storage_->has(other) && this->storage_->state(other) != Invalid);
        this->storage_->allocate(loc);
        // a brand-new matrix: this instance becomes the valid one; otherwise
        // the existing valid instance is copied on first coherent access
        if (fresh && this->storage_->state(loc) == Invalid) this->storage_->modified(loc);
    }

    /// New matrix with the same shape & distribution, no data (Matrix.hh:432).
    Matrix emptyLike(int64_t mb = 0, int64_t nb = 0, Op deepOp = Op::NoTrans) const;

    Matrix sub(int64_t i1, int64_t i2, int64_t j1, int64_t j2) const { return Matrix(BaseMatrix<T>::sub(i1, i2, j1, j2)); }
private:
    void insert_parts(Target target) const;
public:
    Matrix slice(int64_t r1, int64_t r2, int64_t c1, int64_t c2) const { return Matrix(BaseMatrix<T>::slice(r1, r2, c1, c2)); }
};

template <typename T>
class BaseTrapezoidMatrix : public BaseMatrix<T> {
public:
    BaseTrapezoidMatrix() = default;
    BaseTrapezoidMatrix(Uplo uplo, BaseMatrix<T> const& b, MatrixKind k, Diag d = Diag::NonUnit)
        : BaseMatrix<T>(b) {
        slate_error_if_msg(uplo == Uplo::General, "trapezoid matrix requires Upper or Lower");
        // the diagonal of tile (i, i) is the matrix diagonal only for square
        // tiles (reference BaseTrapezoidMatrix.hh:397 asserts tileMb == tileNb)
        slate_error_if_msg(b.mb() != b.nb(), "trapezoid/triangular/Hermitian/symmetric matrix requires square tiles (mb == nb)");
        this->set_uplo(uplo); this->set_kind(k); this->set_diag(d);
    }
    Matrix<T> general() const { Matrix<T> r{BaseMatrix<T>(*this)}; r.set_uplo(Uplo::General); return r; }
};

template <typename T>
class TrapezoidMatrix : public BaseTrapezoidMatrix<T> {
public:
    TrapezoidMatrix() = default;
    TrapezoidMatrix(Uplo uplo, Diag diag, BaseMatrix<T> const& b)
        : BaseTrapezoidMatrix<T>(uplo, b, MatrixKind::Trapezoid, diag) {}
    TrapezoidMatrix(Uplo uplo, Diag diag, int64_t m, int64_t n, int64_t nb, GridPtr g = nullptr)
        : TrapezoidMatrix(uplo, diag, Matrix<T>(m, n, nb, g)) {}
};

template <typename T>
class TriangularMatrix : public BaseTrapezoidMatrix<T> {
public:
    TriangularMatrix() = default;
    TriangularMatrix(Uplo uplo, Diag diag, BaseMatrix<T> const& b)
        : BaseTrapezoidMatrix<T>(uplo, b, MatrixKind::Triangular, diag) {
        slate_error_if_msg(b.m() != b.n(), "triangular matrix must be square");
    }
    TriangularMatrix(Uplo uplo, Diag diag, int64_t n, int64_t nb, GridPtr g = nullptr)
        : TriangularMatrix(uplo, diag, Matrix<T>(n, n, nb, g)) {}
};

template <typename T>
class SymmetricMatrix : public BaseTrapezoidMatrix<T> {
public:
    SymmetricMatrix() = default;
    SymmetricMatrix(Uplo uplo, BaseMatrix<T> const& b)
        : BaseTrapezoidMatrix<T>(uplo, b, MatrixKind::Symmetric) {
        slate_error_if_msg(b.m() != b.n(), "symmetric matrix must be square");
    }
    SymmetricMatrix(Uplo uplo, int64_t n, int64_t nb, GridPtr g = nullptr)
        : SymmetricMatrix(uplo, Matrix<T>(n, n, nb, g)) {}
};

template <typename T>
class HermitianMatrix : public BaseTrapezoidMatrix<T> {
public:
    HermitianMatrix() = default;
    HermitianMatrix(Uplo uplo, BaseMatrix<T> const& b)
        : BaseTrapezoidMatrix<T>(uplo, b, MatrixKind::Hermitian) {
        slate_error_if_msg(b.m() != b.n(), "Hermitian matrix must be square");
    }
    HermitianMatrix(Uplo uplo, int64_t n, int64_t nb, GridPtr g = nullptr)
        : HermitianMatrix(uplo, Matrix<T>(n, n, nb, g)) {}
};

/// General band matrix with lower/upper bandwidths kl/ku.  The sized
/// constructor allocates band-only storage (tiles intersecting the band); a
/// band view of an existing dense matrix keeps that matrix's storage.
template <typename T>
class BandMatrix : public BaseMatrix<T> {
public:
    BandMatrix() = default;
    BandMatrix(int64_t kl, int64_t ku, BaseMatrix<T> const& b) : BaseMatrix<T>(b) {
        this->set_kind(MatrixKind::Band); this->set_band(kl, ku);
    }
    /// (the upper storage bandwidth is ku + kl: room for gbtrf's fill, as
    /// LAPACK's 2 kl + ku + 1 band rows)
    BandMatrix(int64_t m, int64_t n, int64_t kl, int64_t ku, int64_t nb, GridPtr g = nullptr)
        : BandMatrix(kl, ku, Matrix<T>::banded(m, n, kl, ku + kl, nb, g)) {}
    int64_t lowerBandwidth() const { return this->kl(); }
    int64_t upperBandwidth() const { return this->ku(); }
};

template <typename T>
class TriangularBandMatrix : public BaseMatrix<T> {
public:
    TriangularBandMatrix() = default;
    TriangularBandMatrix(Uplo uplo, Diag diag, int64_t kd, BaseMatrix<T> const& b) : BaseMatrix<T>(b) {
        this->set_kind(MatrixKind::TriangularBand); this->set_uplo(uplo); this->set_diag(diag);
        this->set_band(uplo == Uplo::Lower ? kd : 0, uplo == Uplo::Upper ? kd : 0);
    }
    TriangularBandMatrix(Uplo uplo, Diag diag, int64_t n, int64_t kd, int64_t nb, GridPtr g = nullptr)
        : TriangularBandMatrix(uplo, diag, kd, Matrix<T>::banded(n, n, uplo == Uplo::Lower ? kd : 0,
                                                                 uplo == Uplo::Upper ? kd : 0, nb, g)) {}
    int64_t bandwidth() const { return std::max(this->kl(), this->ku()); }
};

template <typename T>
class HermitianBandMatrix : public BaseMatrix<T> {
public:
    HermitianBandMatrix() = default;
    HermitianBandMatrix(Uplo uplo, int64_t kd, BaseMatrix<T> const& b) : BaseMatrix<T>(b) {
        this->set_kind(MatrixKind::HermitianBand); this->set_uplo(uplo);
        this->set_band(uplo == Uplo::Lower ? kd : 0, uplo == Uplo::Upper ? kd : 0);
    }
    HermitianBandMatrix(Uplo uplo, int64_t n, int64_t kd, int64_t nb, GridPtr g = nullptr)
        : HermitianBandMatrix(uplo, kd, Matrix<T>::banded(n, n, uplo == Uplo::Lower ? kd : 0,
                                                          uplo == Uplo::Upper ? kd : 0, nb, g)) {}
    int64_t bandwidth() const { return std::max(this->kl(), this->ku()); }
};

//------------------------------------------------------------------------------
/// Shallow transposes (reference Tile.hh:40-112 / BaseMatrix transpose).
template <typename M> M transpose(M const& A) {
    M r = A;
    static_cast<BaseMatrix<typename M::value_type>&>(r) = A.transpose_view(false);
    return r;
}
template <typename M> M conj_transpose(M const& A) {
    M r = A;
    static_cast<BaseMatrix<typename M::value_type>&>(r) = A.transpose_view(true);
    return r;
}

}  // namespace slate
