// MatrixStorage / BaseMatrix implementation and explicit instantiations.
#include <atomic>
#include "slate_amd/matrix.hh"
#include "slate_amd/inproc.hh"
#include "slate_amd/slate.hh"

#include <complex>
#include <cstring>
#include <cstdlib>

namespace slate {

namespace {
int64_t pad_ld(int64_t mloc, size_t elem) {
    // 256-byte aligned columns, and avoid exact large powers of two (which
    // alias columns onto the same channels/sets).
    int64_t align = std::max<int64_t>(1, 256 / int64_t(elem));
    int64_t ld = roundup(std::max<int64_t>(mloc, 1), align);
    if (ld * int64_t(elem) % 4096 == 0 && ld > 1024) ld += align;
    return ld;
}
}  // namespace

template <typename T>
MatrixStorage<T>::MatrixStorage(int64_t m_, int64_t n_, int64_t mb_, int64_t nb_, GridPtr g,
                                int rsrc_, int csrc_)
    : m(m_), n(n_), mb(mb_), nb(nb_), grid(g), rsrc(rsrc_), csrc(csrc_)
{
    slate_error_if_msg(m < 0 || n < 0, "negative matrix dimension");
    slate_error_if_msg(mb <= 0 || nb <= 0, "tile size must be positive");
    slate_error_if_msg(rsrc < 0 || rsrc >= grid->p() || csrc < 0 || csrc >= grid->q(), "bad rsrc/csrc");
    mloc = numroc(m, mb, rrel(), grid->p());
    nloc = numroc(n, nb, crel(), grid->q());
    lld = pad_ld(mloc, sizeof(T));
}

template <typename T>
MatrixStorage<T>::MatrixStorage(int64_t m_, int64_t n_, std::function<int64_t(int64_t)> const& tile_mb,
                                std::function<int64_t(int64_t)> const& tile_nb,
                                std::function<int(int64_t, int64_t)> const& tile_rank, GridPtr g)
    : m(m_), n(n_), mb(1), nb(1), grid(g), rsrc(0), csrc(0)
{
    slate_error_if_msg(m < 0 || n < 0, "negative matrix dimension");
    auto L = std::make_shared<Layout>();
    L->rs.push_back(0);
    while (L->rs.back() < m) {
        int64_t b = tile_mb(int64_t(L->rs.size()) - 1);
        slate_error_if_msg(b <= 0, "tileMb must be positive");
        L->rs.push_back(std::min(m, L->rs.back() + b));
        mb = std::max(mb, b);
    }
    L->cs.push_back(0);
    while (L->cs.back() < n) {
        int64_t b = tile_nb(int64_t(L->cs.size()) - 1);
        slate_error_if_msg(b <= 0, "tileNb must be positive");
        L->cs.push_back(std::min(n, L->cs.back() + b));
        nb = std::max(nb, b);
    }
    L->mt = int64_t(L->rs.size()) - 1;
    L->nt = int64_t(L->cs.size()) - 1;
    L->owner.resize(size_t(L->mt * L->nt));
    L->toff.assign(size_t(L->mt * L->nt), -1);
    int64_t off = 0;
    const int me = g->rank();
    for (int64_t j = 0; j < L->nt; ++j)
        for (int64_t i = 0; i < L->mt; ++i) {
            int r = tile_rank(i, j);
            slate_error_if_msg(r < 0 || r >= g->size(), "tileRank out of range");
            L->owner[i + j * L->mt] = r;
            if (r == me) {
                L->toff[i + j * L->mt] = off;
                off += (L->rs[i + 1] - L->rs[i]) * (L->cs[j + 1] - L->cs[j]);
            }
        }
    layout = L;
    // the packed local tiles as one column (allocate / copy_instance unchanged)
    mloc = off;
    nloc = off > 0 ? 1 : 0;
    lld = std::max<int64_t>(off, 1);
}

template <typename T>
MatrixStorage<T>::MatrixStorage(int64_t m_, int64_t n_, int64_t nb_, GridPtr g, int64_t kl, int64_t ku, BandTag)
    : MatrixStorage(m_, n_, nb_, nb_, g, 0, 0)
{
    slate_error_if_msg(kl < 0 || ku < 0, "band matrix: negative bandwidth");
    banded = true;
    band_lt = ceildiv(kl, nb);
    band_ut = ceildiv(ku, nb);
    const int64_t mt = ceildiv(m, mb), ntl = ceildiv(nloc, nb);
    const int p = grid->p(), q = grid->q();
    boff.assign(ntl, 0);
    bend.assign(ntl, 0);
    int64_t h = 0;
    for (int64_t lj = 0; lj < ntl; ++lj) {
        const int64_t J = lj * q + crel();
        const int64_t i_lo = std::max<int64_t>(0, J - band_ut), i_hi = std::min<int64_t>(mt - 1, J + band_lt);
        if (i_lo > i_hi) { boff[lj] = bend[lj] = 0; continue; }
        boff[lj] = numroc(i_lo * mb, mb, rrel(), p);
        bend[lj] = numroc(std::min(m, (i_hi + 1) * mb), mb, rrel(), p);
        h = std::max(h, bend[lj] - boff[lj]);
    }
    lld = pad_ld(h, sizeof(T));
}

template <typename T>
MatrixStorage<T>::~MatrixStorage() {
    for (auto& kv : ws_tiles) {
        if (kv.second.loc == Loc::Host) std::free(kv.second.ptr);
        else { try { device::free(kv.second.ptr); } catch (...) {} }
    }
    if (host_owned_ && host_) std::free(host_);
    if (dev_owned_ && dev_) {
        try { device::free(dev_); } catch (...) {}
    }
}

template <typename T>
void MatrixStorage<T>::attach(T* ptr, int64_t ld_, Loc loc) {
    slate_error_if_msg(ld_ < std::max<int64_t>(1, mloc), "leading dimension too small");
    if (loc == Loc::Host) {
        slate_assert(!host_);
        host_ = ptr; host_ld_ = ld_; host_owned_ = false; host_state_ = Modified;
        if (dev_) dev_state_ = Invalid;
    } else {
        slate_assert(!dev_);
        dev_ = ptr; dev_ld_ = ld_; dev_owned_ = false; dev_state_ = Modified;
        if (host_) host_state_ = Invalid;
    }
    origin_ = loc;
    kind_ = TileKind::UserOwned;
}

namespace {
std::atomic<size_t> g_storage_max{0};
}
size_t storage_alloc_max() { return g_storage_max.load(); }
void storage_alloc_reset() { g_storage_max.store(0); }

template <typename T>
void MatrixStorage<T>::allocate(Loc loc) {
    slate_error_if_msg(multi(), "multi-device matrix: no caller-side local array (drivers run on its devices; "
                                "Matrix::gather copies it out)");
    size_t bytes = size_t(lld) * size_t(std::max<int64_t>(nloc, 1)) * sizeof(T);
    if ((loc == Loc::Host ? host_ : dev_) == nullptr) {
        size_t cur = g_storage_max.load();
        while (bytes > cur && !g_storage_max.compare_exchange_weak(cur, bytes)) {}
    }
    if (loc == Loc::Host) {
        if (host_) return;
        void* p = nullptr;
        if (posix_memalign(&p, 256, std::max<size_t>(bytes, 256)) != 0) throw std::bad_alloc();
        host_ = static_cast<T*>(p);
        host_ld_ = lld; host_owned_ = true;
        if (!dev_) origin_ = Loc::Host;
    } else {
        if (dev_) return;
        dev_ = static_cast<T*>(device::malloc(std::max<size_t>(bytes, 256)));
        dev_ld_ = lld; dev_owned_ = true;
        if (!host_) origin_ = Loc::Device;
    }
}

template <typename T>
void MatrixStorage<T>::copy_instance(Loc to) {
    T* src = to == Loc::Host ? dev_ : host_;
    T* dst = to == Loc::Host ? host_ : dev_;
    int64_t sld = to == Loc::Host ? dev_ld_ : host_ld_;
    int64_t dld = to == Loc::Host ? host_ld_ : dev_ld_;
    if (mloc == 0 || nloc == 0) return;
    const int64_t rows = banded ? lld : mloc;     // band-only storage: the whole band array
    hipStream_t s = device::queue(0);
    device::memcpy2d_async(dst, dld * sizeof(T), src, sld * sizeof(T), rows * sizeof(T), nloc, s);
    slate_hip_call(hipStreamSynchronize(s));
}

template <typename T>
T* MatrixStorage<T>::get(Loc loc, bool for_write) {
    allocate(loc);
    MOSI_State& mine  = loc == Loc::Host ? host_state_ : dev_state_;
    MOSI_State& other = loc == Loc::Host ? dev_state_ : host_state_;
    if (mine == Invalid) {
        if (other != Invalid && has(loc == Loc::Host ? Loc::Device : Loc::Host)) {
            copy_instance(loc);
            if (other == Modified) other = Shared;
        }
        mine = Shared;
    }
    if (for_write) {
        mine = Modified;
        if (has(loc == Loc::Host ? Loc::Device : Loc::Host)) other = Invalid;
    }
    return raw(loc);
}

template <typename T>
void MatrixStorage<T>::modified(Loc loc) {
    allocate(loc);
    (loc == Loc::Host ? host_state_ : dev_state_) = Modified;
    Loc o = loc == Loc::Host ? Loc::Device : Loc::Host;
    if (has(o)) (o == Loc::Host ? host_state_ : dev_state_) = Invalid;
}

template <typename T>
void MatrixStorage<T>::update_origin() {
    if (state(origin_) == Invalid) get(origin_, false);
}

template <typename T>
void MatrixStorage<T>::release_workspace() {
    Loc o = origin_ == Loc::Host ? Loc::Device : Loc::Host;
    if (!has(o)) return;
    update_origin();
    if (o == Loc::Device && dev_owned_) { device::free(dev_); dev_ = nullptr; dev_state_ = Invalid; dev_owned_ = false; }
    if (o == Loc::Host && host_owned_)  { std::free(host_); host_ = nullptr; host_state_ = Invalid; host_owned_ = false; }
}

//------------------------------------------------------------------------------
template <typename T>
BaseMatrix<T> BaseMatrix<T>::sub(int64_t i1, int64_t i2, int64_t j1, int64_t j2) const {
    // logical -> storage tile ranges
    int64_t si1, si2, sj1, sj2;
    if (op_ == Op::NoTrans) { si1 = i1; si2 = i2; sj1 = j1; sj2 = j2; }
    else { si1 = j1; si2 = j2; sj1 = i1; sj2 = i2; }
    slate_error_if_msg(storage_->general() && !(si1 == 0 && sj1 == 0 && si2 == smt() - 1 && sj2 == snt() - 1),
                       "sub: views of an arbitrary-distribution matrix are whole-matrix only");
    BaseMatrix r = *this;
    // empty ranges allowed (i2 = i1 - 1)
    slate_error_if_msg(si1 < 0 || sj1 < 0 || si2 >= std::max<int64_t>(smt(), si1) ||
                       sj2 >= std::max<int64_t>(snt(), sj1), "sub: tile index out of range");
    if (si2 < si1) { r.r0_ = si1 < smt() ? srow_start(si1) : r0_ + m_; r.m_ = 0; }
    else { r.r0_ = srow_start(si1); r.m_ = srow_start(si2) + srow_size(si2) - r.r0_; }
    if (sj2 < sj1) { r.c0_ = sj1 < snt() ? scol_start(sj1) : c0_ + n_; r.n_ = 0; }
    else { r.c0_ = scol_start(sj1); r.n_ = scol_start(sj2) + scol_size(sj2) - r.c0_; }
    // a sub-matrix that is off the diagonal is general
    if (!(si1 == sj1 && si2 == sj2)) {
        if (kind_ == MatrixKind::Symmetric || kind_ == MatrixKind::Hermitian ||
            kind_ == MatrixKind::Triangular || kind_ == MatrixKind::Trapezoid) {
            // keep uplo for diagonal-touching views; callers re-wrap as needed
        }
    }
    return r;
}

template <typename T>
BaseMatrix<T> BaseMatrix<T>::slice(int64_t r1, int64_t r2, int64_t c1, int64_t c2) const {
    int64_t sr1, sr2, sc1, sc2;
    if (op_ == Op::NoTrans) { sr1 = r1; sr2 = r2; sc1 = c1; sc2 = c2; }
    else { sr1 = c1; sr2 = c2; sc1 = r1; sc2 = r2; }
    slate_error_if_msg(sr1 < 0 || sc1 < 0 || sr2 >= m_ || sc2 >= n_ || sr2 < sr1 - 1 || sc2 < sc1 - 1,
                       "slice: index out of range");
    slate_error_if_msg(storage_->general() && !(sr1 == 0 && sc1 == 0 && sr2 == m_ - 1 && sc2 == n_ - 1),
                       "slice: views of an arbitrary-distribution matrix are whole-matrix only");
    BaseMatrix r = *this;
    r.r0_ = r0_ + sr1; r.m_ = sr2 - sr1 + 1;
    r.c0_ = c0_ + sc1; r.n_ = sc2 - sc1 + 1;
    return r;
}

template <typename T>
int64_t BaseMatrix<T>::lrow_begin() const {
    return g2l_ceil(r0_, storage_->mb, storage_->rrel(), storage_->grid->p());
}
template <typename T>
int64_t BaseMatrix<T>::lrow_end() const {
    return g2l_ceil(r0_ + m_, storage_->mb, storage_->rrel(), storage_->grid->p());
}
template <typename T>
int64_t BaseMatrix<T>::lcol_begin() const {
    return g2l_ceil(c0_, storage_->nb, storage_->crel(), storage_->grid->q());
}
template <typename T>
int64_t BaseMatrix<T>::lcol_end() const {
    return g2l_ceil(c0_ + n_, storage_->nb, storage_->crel(), storage_->grid->q());
}

template <typename T>
LocalBlock<T> BaseMatrix<T>::local_raw(Loc loc) const {
    slate_error_if_msg(storage_->general(),
                       "arbitrary-distribution matrix: no block-cyclic local array (copy / redistribute it into a "
                       "block-cyclic Matrix, as the drivers do)");
    slate_error_if_msg(storage_->banded,
                       "band-only storage: no dense local array (band drivers read it tile column by tile column)");
    slate_error_if_msg(storage_->multi(),
                       "multi-device matrix: this operation does not run on multi-device matrices (gather it, or "
                       "use a driver that accepts them, see Matrix::multiDevice)");
    LocalBlock<T> b;
    int64_t rb = lrow_begin(), re = lrow_end(), cb = lcol_begin(), ce = lcol_end();
    b.m = re - rb; b.n = ce - cb;
    b.ld = std::max<int64_t>(1, storage_->ld(loc));
    T* base = storage_->raw(loc);
    b.ptr = base ? base + rb + cb * b.ld : nullptr;
    return b;
}

template <typename T>
LocalBlock<T> BaseMatrix<T>::local(Loc loc, bool for_write) const {
    storage_->get(loc, for_write);
    return local_raw(loc);
}

template <typename T>
Tile<T> BaseMatrix<T>::tile(int64_t i, int64_t j, Loc loc) const {
    int64_t si, sj; to_storage(i, j, si, sj);
    if (!tileIsLocal(i, j)) {
        // a remote tile received into workspace (tile_comm.cc)
        auto it = storage_->ws_tiles.find(skey(si, sj));
        slate_error_if_msg(it == storage_->ws_tiles.end(), "tile: not local (and not received)");
        auto const& w = it->second;
        slate_error_if_msg(w.loc != loc, "tile: the received tile lives at the other location");
        Tile<T> t;
        t.data = w.ptr; t.mb = w.mb; t.nb = w.nb;
        auto lt = storage_->tile_layouts.find(skey(si, sj));
        t.layout = lt == storage_->tile_layouts.end() ? Layout::ColMajor : lt->second;
        t.stride = std::max<int64_t>(1, t.layout == Layout::ColMajor ? w.mb : w.nb);
        t.op = op_; t.uplo = uplo_physical();
        t.device = loc == Loc::Host ? HostNum : 0;
        return t;
    }
    if (storage_->general()) {
        auto const& L = *storage_->layout;
        T* base = storage_->raw(loc);
        slate_error_if_msg(!base, "tile: storage not allocated at location");
        Tile<T> t;
        t.mb = srow_size(si); t.nb = scol_size(sj); t.stride = std::max<int64_t>(t.mb, 1);
        t.data = base + L.toff[si + sj * L.mt];
        t.op = op_; t.uplo = uplo_physical();
        t.device = loc == Loc::Host ? HostNum : 0;
        auto lt = storage_->tile_layouts.find(skey(si, sj));
        if (lt != storage_->tile_layouts.end()) t.layout = lt->second;
        return t;
    }
    auto& g = *storage_->grid;
    int64_t gr = srow_start(si), gc = scol_start(sj);
    int64_t lr = g2l(gr, storage_->mb, g.p()), lc = g2l(gc, storage_->nb, g.q());
    Tile<T> t;
    int64_t ld = storage_->ld(loc);
    T* base = storage_->raw(loc);
    slate_error_if_msg(!base, "tile: storage not allocated at location");
    t.data = storage_->banded ? storage_->local_ptr(loc, lr, lc) : base + lr + lc * ld;
    slate_error_if_msg(!t.data, "tile: outside the stored band");
    t.mb = srow_size(si); t.nb = scol_size(sj); t.stride = ld;
    t.op = op_; t.uplo = uplo_physical();
    t.device = loc == Loc::Host ? HostNum : 0;
    if (!storage_->tile_layouts.empty()) {
        auto lt = storage_->tile_layouts.find(skey(si, sj));
        if (lt != storage_->tile_layouts.end()) t.layout = lt->second;
    }
    return t;
}

template <typename T>
T& BaseMatrix<T>::elem(int64_t i, int64_t j) {
    int64_t si = op_ == Op::NoTrans ? i : j, sj = op_ == Op::NoTrans ? j : i;
    int64_t gr = r0_ + si, gc = c0_ + sj;
    auto& g = *storage_->grid;
    slate_error_if_msg(storage_->row_owner(gr / storage_->mb) != g.myrow() ||
                       storage_->col_owner(gc / storage_->nb) != g.mycol(), "elem: not local");
    storage_->get(Loc::Host, false);
    T* e = storage_->local_ptr(Loc::Host, g2l(gr, storage_->mb, g.p()), g2l(gc, storage_->nb, g.q()));
    slate_error_if_msg(!e, "elem: outside the stored band");
    return *e;
}

//------------------------------------------------------------------------------
template <typename T>
Matrix<T> Matrix<T>::fromLAPACK(int64_t m, int64_t n, T* A, int64_t lda, int64_t nb, Loc loc) {
    Matrix<T> M(m, n, nb, nb, Grid::self());
    M.storage_->attach(A, lda, loc);
    return M;
}

template <typename T>
Matrix<T> Matrix<T>::fromScaLAPACK(int64_t m, int64_t n, T* A, int64_t lld, int64_t mb, int64_t nb,
                                   GridPtr grid, Loc loc, int rsrc, int csrc) {
    Matrix<T> M(m, n, mb, nb, grid ? grid : default_grid(), rsrc, csrc);
    M.storage_->attach(A, lld, loc);
    return M;
}

namespace {
/// caller-side storage of a multi-device matrix on `group`, with parts
template <typename T>
std::shared_ptr<MatrixStorage<T>> multi_storage(int64_t m, int64_t n, int64_t mb, int64_t nb,
                                                std::shared_ptr<InprocGroup> const& group,
                                                std::vector<std::shared_ptr<MatrixStorage<T>>> parts) {
    auto st = std::make_shared<MatrixStorage<T>>(m, n, mb, nb, Grid::self());
    st->group = group;
    st->parts = std::move(parts);
    return st;
}
}  // namespace

template <typename T>
Matrix<T> Matrix<T>::fromDevices(int64_t m, int64_t n, T** Aarray, int num_devices, int64_t lda, int64_t mb,
                                 int64_t nb, int p, int q) {
    slate_error_if_msg(p * q != 1, "fromDevices(Aarray, num_devices): one process drives its devices (p = q = 1); "
                                   "a p x q job runs one GPU per process");
    slate_error_if_msg(num_devices < 1 || !Aarray, "fromDevices: num_devices >= 1 arrays required");
    const bool dev = device::available();
    // array d lives on device d (d mod the device count when fewer GPUs are
    // visible: ranks then share one, as in the one-GPU tests)
    std::vector<int> devs;
    if (dev) for (int d = 0; d < num_devices; ++d) devs.push_back(d % device::count());
    // tile column j on device j % num_devices: a 1 x num_devices group
    auto group = InprocGroup::get(1, num_devices, devs, GridOrder::Col);
    std::vector<std::shared_ptr<MatrixStorage<T>>> parts;
    for (int r = 0; r < num_devices; ++r) {
        auto ps = std::make_shared<MatrixStorage<T>>(m, n, mb, nb, group->grid(r));
        ps->attach(Aarray[r], lda, dev ? Loc::Device : Loc::Host);
        parts.push_back(ps);
    }
    return Matrix<T>(BaseMatrix<T>(multi_storage<T>(m, n, mb, nb, group, std::move(parts))));
}

template <typename T>
Matrix<T> Matrix<T>::multiDevice(int64_t m, int64_t n, int64_t mb, int64_t nb, int num_devices) {
    auto group = InprocGroup::of_size(num_devices);
    std::vector<std::shared_ptr<MatrixStorage<T>>> parts;
    for (int r = 0; r < group->size(); ++r)
        parts.push_back(std::make_shared<MatrixStorage<T>>(m, n, mb, nb, group->grid(r)));
    Matrix<T> M(BaseMatrix<T>(multi_storage<T>(m, n, mb, nb, group, std::move(parts))));
    M.insertLocalTiles(Target::Devices);
    return M;
}

template <typename T>
Matrix<T> Matrix<T>::fromParts(std::shared_ptr<InprocGroup> const& group, std::vector<Matrix<T>> const& parts) {
    slate_error_if_msg(!group || int(parts.size()) != group->size(), "fromParts: one matrix per rank");
    std::vector<std::shared_ptr<MatrixStorage<T>>> st;
    for (auto const& P : parts) {
        slate_error_if_msg(!P.storage(), "fromParts: empty part");
        st.push_back(P.storage());
    }
    auto const& p0 = *st[0];
    Matrix<T> M(BaseMatrix<T>(multi_storage<T>(p0.m, p0.n, p0.mb, p0.nb, group, std::move(st))));
    // the view of part 0 (offsets, op, uplo, ...) on the caller-side storage
    BaseMatrix<T> v = parts[0];
    static_cast<BaseMatrix<T>&>(M) = M.rebase(v);
    return M;
}

template <typename T>
void Matrix<T>::insert_parts(Target target) const {
    auto& st = *this->storage_;
    // each rank allocates its part in its own device context
    const Target t = device::available() ? target : Target::Host;
    st.group->run([&](int r, GridPtr const&) {
        Matrix<T>(BaseMatrix<T>(st.parts[size_t(r)])).insertLocalTiles(t);
    });
}

template <typename T>
void Matrix<T>::gather(T* A, int64_t lda) const {
    slate_error_if_msg(lda < std::max<int64_t>(1, this->m()), "gather: lda < m");
    auto copy_out = [&](std::vector<T> const& full) {
        const int64_t m = this->m(), n = this->n();
        for (int64_t j = 0; j < n; ++j) std::memcpy(A + j * lda, full.data() + j * m, size_t(m) * sizeof(T));
    };
    if (!this->is_multi_device()) {
        std::vector<T> full;
        slate::gather(BaseMatrix<T>(*this), full);
        copy_out(full);
        return;
    }
    std::vector<T> full;
    this->storage_->group->run([&](int r, GridPtr const&) {
        std::vector<T> f;
        slate::gather(this->on_part(r), f);
        if (r == 0) full.swap(f);
    });
    copy_out(full);
}

template <typename T>
Matrix<T> Matrix<T>::emptyLike(int64_t mb, int64_t nb, Op deepOp) const {
    if (this->is_multi_device()) {
        auto& st = *this->storage_;
        std::vector<std::shared_ptr<MatrixStorage<T>>> parts;
        for (int r = 0; r < st.group->size(); ++r)
            parts.push_back(Matrix<T>(this->on_part(r)).emptyLike(mb, nb, deepOp).storage());
        auto const& p0 = *parts[0];
        return Matrix<T>(BaseMatrix<T>(multi_storage<T>(p0.m, p0.n, p0.mb, p0.nb, st.group, std::move(parts))));
    }
    // New storage over the same logical tile grid as this view, with the
    // first tile on the same rank (so tiles (i, j) of both are co-located).
    slate_error_if_msg(!this->aligned(), "emptyLike: view must start on a tile boundary");
    int64_t mt = this->mt(), nt = this->nt();
    GridPtr g = this->storage_->grid;
    int64_t tmb = this->op_ == Op::NoTrans ? this->storage_->mb : this->storage_->nb;
    int64_t tnb = this->op_ == Op::NoTrans ? this->storage_->nb : this->storage_->mb;
    int64_t m_l = this->m(), n_l = this->n();
    if (this->op_ != Op::NoTrans) g = g->transposed();
    int r00 = mt > 0 && nt > 0 ? this->tileRank(0, 0) : this->mpiRank();
    int rsrc = g->row_of(r00), csrc = g->col_of(r00);
    if (mb > 0) { tmb = mb; m_l = mt * mb; }
    if (nb > 0) { tnb = nb; n_l = nt * nb; }
    if (deepOp != Op::NoTrans) {
        std::swap(m_l, n_l); std::swap(tmb, tnb); std::swap(rsrc, csrc);
        g = g->transposed();
    }
    return Matrix<T>(m_l, n_l, tmb, tnb, g, rsrc, csrc);
}

//------------------------------------------------------------------------------
template class MatrixStorage<float>;
template class MatrixStorage<double>;
template class MatrixStorage<std::complex<float>>;
template class MatrixStorage<std::complex<double>>;
template class BaseMatrix<float>;
template class BaseMatrix<double>;
template class BaseMatrix<std::complex<float>>;
template class BaseMatrix<std::complex<double>>;
template class Matrix<float>;
template class Matrix<double>;
template class Matrix<std::complex<float>>;
template class Matrix<std::complex<double>>;

}  // namespace slate
