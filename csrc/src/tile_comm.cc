// Tile-level communication and layout conversion (reference
// include/slate/Tile.hh:813-1270 send / recv / bcast / layoutConvert and
// BaseMatrix.hh tileSend / tileRecv / tileBcast / tileBcastToSet /
// tileLayoutConvert).
//
// Here a tile is a strided block of the process's contiguous local array (or,
// for a remote tile, a contiguous workspace buffer in the matrix storage), so
// a message is the tile packed column-major into one buffer and moved by the
// grid's world communicator: RCCL send / recv on the device (stream ordered,
// over xGMI peer links), the native TCP mesh or the in-process transport on
// the host.  Broadcasts are binomial trees of point-to-point messages rooted
// at the owner, so a set of k ranks takes ceil(log2 k) message rounds.
#include "internal.hh"

#include <algorithm>
#include <cstdlib>

namespace slate {

using internal::Work;

template <typename T>
T* MatrixStorage<T>::ws_tile(int64_t si, int64_t sj, int64_t mb_, int64_t nb_, Loc loc) {
    const auto key = std::make_pair(si, sj);
    auto it = ws_tiles.find(key);
    if (it != ws_tiles.end()) {
        if (it->second.loc == loc && it->second.mb == mb_ && it->second.nb == nb_) return it->second.ptr;
        ws_erase(si, sj);
    }
    WsTile w;
    w.mb = mb_; w.nb = nb_; w.loc = loc;
    const size_t bytes = size_t(std::max<int64_t>(mb_ * nb_, 1)) * sizeof(T);
    w.ptr = static_cast<T*>(loc == Loc::Host ? std::malloc(bytes) : device::malloc(bytes));
    slate_error_if_msg(!w.ptr, "workspace tile: out of memory");
    ws_tiles[key] = w;
    return w.ptr;
}

template <typename T>
void MatrixStorage<T>::ws_erase(int64_t si, int64_t sj) {
    const auto key = std::make_pair(si, sj);
    auto it = ws_tiles.find(key);
    if (it == ws_tiles.end()) return;
    if (it->second.loc == Loc::Host) std::free(it->second.ptr);
    else device::free(it->second.ptr);
    ws_tiles.erase(it);
    tile_layouts.erase(key);
}

namespace {

/// where tile messages of this matrix live: the device instance when it is
/// the valid one (or both are), else the host
template <typename T>
Loc msg_loc(MatrixStorage<T> const& st) {
    if (st.raw(Loc::Device) && st.state(Loc::Device) != Invalid) return Loc::Device;
    return Loc::Host;
}

template <typename T>
lb::Ctx msg_ctx(Loc loc) {
    return loc == Loc::Device ? lb::Ctx::device(0) : lb::Ctx::host();
}

/// tile (stored mb x nb, `layout`) -> contiguous column-major buffer
template <typename T>
void pack_tile(lb::Ctx const& c, Tile<T> const& t, T* buf) {
    if (t.layout == Layout::ColMajor) lb::copy2d(c, t.mb, t.nb, t.data, t.stride, buf, std::max<int64_t>(t.mb, 1));
    else lb::copy<T, T>(c, Uplo::General, Op::Trans, t.mb, t.nb, t.data, t.stride, buf, std::max<int64_t>(t.mb, 1));
}

/// contiguous column-major buffer -> tile storage (column-major)
template <typename T>
void unpack_tile(lb::Ctx const& c, T const* buf, Tile<T> const& t) {
    lb::copy2d(c, t.mb, t.nb, buf, std::max<int64_t>(t.mb, 1), t.data, t.stride);
}

template <typename T>
void sync_ctx(lb::Ctx const& c) {
    if (c.dev()) slate_hip_call(hipStreamSynchronize(c.stream));
}

}  // namespace

template <typename T>
bool BaseMatrix<T>::tileExists(int64_t i, int64_t j) const {
    if (tileIsLocal(i, j)) return true;
    int64_t si, sj; to_storage(i, j, si, sj);
    return storage_->ws_tiles.count(skey(si, sj)) > 0;
}

template <typename T>
Layout BaseMatrix<T>::tileLayout(int64_t i, int64_t j) const {
    int64_t si, sj; to_storage(i, j, si, sj);
    auto it = storage_->tile_layouts.find(skey(si, sj));
    return it == storage_->tile_layouts.end() ? Layout::ColMajor : it->second;
}

template <typename T>
void BaseMatrix<T>::tileSend(int64_t i, int64_t j, int dst_rank, int tag) const {
    (void)tag;
    slate_error_if_msg(!tileExists(i, j), "tileSend: tile neither local nor received");
    Comm& w = grid()->world();
    const Loc loc = msg_loc(*storage_);
    if (tileIsLocal(i, j)) storage_->get(loc, false);
    Tile<T> t = tile(i, j, loc);
    lb::Ctx c = msg_ctx<T>(loc);
    const size_t cnt = size_t(t.mb) * t.nb;
    Work<T> buf(loc == Loc::Device ? Target::Devices : Target::HostTask, std::max<size_t>(cnt, 1));
    pack_tile(c, t, buf.data());
    w.exchange({{buf.data(), cnt, dst_rank, true}}, scalar_type<T>(), loc, c.stream);
    sync_ctx<T>(c);
}

template <typename T>
void BaseMatrix<T>::tileRecv(int64_t i, int64_t j, int src_rank, Layout layout, int tag) {
    (void)tag;
    Comm& w = grid()->world();
    const Loc loc = msg_loc(*storage_);
    int64_t si, sj; to_storage(i, j, si, sj);
    const int64_t mb_ = srow_size(si), nb_ = scol_size(sj);
    if (tileIsLocal(i, j)) storage_->get(loc, true);
    else {
        storage_->ws_tile(skey(si, sj).first, skey(si, sj).second, mb_, nb_, loc);
        storage_->tile_layouts.erase(skey(si, sj));
    }
    if (tileIsLocal(i, j)) storage_->tile_layouts.erase(skey(si, sj));
    Tile<T> t = tile(i, j, loc);
    lb::Ctx c = msg_ctx<T>(loc);
    const size_t cnt = size_t(mb_) * nb_;
    Work<T> buf(loc == Loc::Device ? Target::Devices : Target::HostTask, std::max<size_t>(cnt, 1));
    w.exchange({{buf.data(), cnt, src_rank, false}}, scalar_type<T>(), loc, c.stream);
    unpack_tile(c, buf.data(), t);
    sync_ctx<T>(c);
    if (tileIsLocal(i, j)) storage_->modified(loc);
    if (layout == Layout::RowMajor) tileLayoutConvert(i, j, Layout::RowMajor);
}

template <typename T>
void BaseMatrix<T>::tileBcastToSet(int64_t i, int64_t j, std::set<int> const& ranks, Layout layout) {
    const int root = tileRank(i, j), me = mpiRank();
    std::vector<int> order = {root};
    for (int r : ranks) if (r != root) order.push_back(r);
    const int n = int(order.size());
    const int pos = int(std::find(order.begin(), order.end(), me) - order.begin());
    if (pos >= n) return;   // not a participant
    // binomial tree: in round `mask`, positions < mask send to pos + mask
    for (int mask = 1; mask < n; mask <<= 1) {
        if (pos < mask) {
            if (pos + mask < n) tileSend(i, j, order[pos + mask]);
        } else if (pos < 2 * mask) {
            tileRecv(i, j, order[pos - mask], Layout::ColMajor);
        }
    }
    if (pos > 0 && layout == Layout::RowMajor) tileLayoutConvert(i, j, Layout::RowMajor);
}

template <typename T>
void BaseMatrix<T>::tileBcast(int64_t i, int64_t j, BaseMatrix<T> const& B, Layout layout, int tag) {
    (void)tag;
    std::set<int> ranks;
    for (int64_t bi = 0; bi < B.mt(); ++bi)
        for (int64_t bj = 0; bj < B.nt(); ++bj) ranks.insert(B.tileRank(bi, bj));
    tileBcastToSet(i, j, ranks, layout);
}

template <typename T>
void BaseMatrix<T>::tileLayoutConvert(int64_t i, int64_t j, Layout layout) {
    if (tileLayout(i, j) == layout) return;
    int64_t si, sj; to_storage(i, j, si, sj);
    const auto key = skey(si, sj);
    const bool local = tileIsLocal(i, j);
    Loc loc;
    if (local) {
        loc = msg_loc(*storage_);
        storage_->get(loc, true);
    } else {
        auto it = storage_->ws_tiles.find(key);
        slate_error_if_msg(it == storage_->ws_tiles.end(), "tileLayoutConvert: tile neither local nor received");
        loc = it->second.loc;
    }
    Tile<T> t = tile(i, j, loc);
    // stored block: rows x cols with leading dimension t.stride
    const int64_t rows = t.layout == Layout::ColMajor ? t.mb : t.nb;
    const int64_t cols = t.layout == Layout::ColMajor ? t.nb : t.mb;
    slate_error_if_msg(rows != cols && local,
                       "tileLayoutConvert: rectangular tiles convert only as contiguous (received) tiles");
    lb::Ctx c = msg_ctx<T>(loc);
    const size_t cnt = size_t(rows) * cols;
    Work<T> tmp(loc == Loc::Device ? Target::Devices : Target::HostTask, std::max<size_t>(cnt, 1));
    // transpose into tmp (cols x rows, contiguous), then back over the block
    lb::copy<T, T>(c, Uplo::General, Op::Trans, cols, rows, t.data, t.stride, tmp.data(), std::max<int64_t>(cols, 1));
    const int64_t ld_new = local ? t.stride : std::max<int64_t>(cols, 1);
    lb::copy2d(c, cols, rows, tmp.data(), std::max<int64_t>(cols, 1), t.data, ld_new);
    sync_ctx<T>(c);
    if (local) storage_->modified(loc);
    if (layout == Layout::ColMajor) storage_->tile_layouts.erase(key);
    else storage_->tile_layouts[key] = layout;
}

template <typename T>
void BaseMatrix<T>::tileLayoutReset() {
    std::vector<std::pair<int64_t, int64_t>> keys;
    for (auto const& kv : storage_->tile_layouts) keys.push_back(kv.first);
    for (auto const& k : keys) {
        if (storage_->ws_tiles.count(k)) continue;
        // absolute storage tile -> logical tile of the full-storage view
        BaseMatrix<T> full(storage_);
        full.tileLayoutConvert(k.first, k.second, Layout::ColMajor);
    }
}

template <typename T>
void BaseMatrix<T>::tileErase(int64_t i, int64_t j) {
    if (tileIsLocal(i, j)) return;
    int64_t si, sj; to_storage(i, j, si, sj);
    const auto k = skey(si, sj);
    storage_->ws_erase(k.first, k.second);
}

#define SLATE_TILE_COMM_INST(T)                                                                         \
    template T* MatrixStorage<T>::ws_tile(int64_t, int64_t, int64_t, int64_t, Loc);                    \
    template void MatrixStorage<T>::ws_erase(int64_t, int64_t);                                         \
    template bool BaseMatrix<T>::tileExists(int64_t, int64_t) const;                                    \
    template Layout BaseMatrix<T>::tileLayout(int64_t, int64_t) const;                                  \
    template void BaseMatrix<T>::tileSend(int64_t, int64_t, int, int) const;                            \
    template void BaseMatrix<T>::tileRecv(int64_t, int64_t, int, Layout, int);                          \
    template void BaseMatrix<T>::tileBcastToSet(int64_t, int64_t, std::set<int> const&, Layout);        \
    template void BaseMatrix<T>::tileBcast(int64_t, int64_t, BaseMatrix<T> const&, Layout, int);        \
    template void BaseMatrix<T>::tileLayoutConvert(int64_t, int64_t, Layout);                           \
    template void BaseMatrix<T>::tileLayoutReset();                                                     \
    template void BaseMatrix<T>::tileErase(int64_t, int64_t);

SLATE_TILE_COMM_INST(float)
SLATE_TILE_COMM_INST(double)
SLATE_TILE_COMM_INST(std::complex<float>)
SLATE_TILE_COMM_INST(std::complex<double>)

}  // namespace slate
