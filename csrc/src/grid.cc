#include "slate_amd/grid.hh"

#include <mutex>

namespace slate {

Grid::Grid(int p, int q, GridOrder order, CommPtr world, CommPtr row, CommPtr col)
    : p_(p), q_(q), order_(order), world_(world), row_(row), col_(col)
{
    slate_assert(p >= 1 && q >= 1);
    slate_assert(order == GridOrder::Col || order == GridOrder::Row);
    slate_error_if_msg(world_->size() != p * q, "grid: world size != p*q");
    myrow_ = row_of(world_->rank());
    mycol_ = col_of(world_->rank());
    slate_error_if_msg(row_->size() != q || col_->size() != p, "grid: row/col comm sizes");
    slate_error_if_msg(row_->rank() != mycol_ || col_->rank() != myrow_,
                       "grid: row comm rank must be the process column, col comm rank the process row");
}

std::shared_ptr<Grid> Grid::self() {
    static std::shared_ptr<Grid> g = [] {
        auto c = std::make_shared<SelfComm>();
        return std::make_shared<Grid>(1, 1, GridOrder::Col, c, c, c);
    }();
    return g;
}

std::shared_ptr<Grid> Grid::transposed() const {
    // (r, c) on this grid  ->  (c, r) on a q x p grid with the opposite order
    GridOrder o = order_ == GridOrder::Col ? GridOrder::Row : GridOrder::Col;
    auto t = std::make_shared<Grid>(q_, p_, o, world_, col_, row_);
    if (has_fast_lane()) t->set_fast(col_fast_ptr(), row_fast_ptr());
    return t;
}

namespace {
std::mutex g_mtx;
GridPtr g_default;
}

thread_local GridPtr t_default;

GridPtr default_grid() {
    if (t_default) return t_default;
    std::lock_guard<std::mutex> l(g_mtx);
    return g_default ? g_default : Grid::self();
}

void set_thread_default_grid(GridPtr g) { t_default = std::move(g); }

void set_default_grid(GridPtr g) {
    std::lock_guard<std::mutex> l(g_mtx);
    g_default = g;
}

}  // namespace slate
