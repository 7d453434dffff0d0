// pybind11 bindings for the native library (module slate_d35_amd._slate).
//
// Exposes the process grid / communicators, the distributed matrix classes,
// DLPack export of device-resident local arrays (zero-copy into torch), and
// every driver.  The GIL is released while drivers run; host communicators
// implemented in Python (torch.distributed / gloo) re-acquire it through the
// trampoline below.
#include <pybind11/pybind11.h>
#include <chrono>
#include <thread>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>
#include <pybind11/functional.h>

#include "slate_amd/slate.hh"
#include "../src/lu_dist.hh"
#include "slate_amd/trace.hh"
#include "slate_amd/runtime.hh"
#include "slate_amd/inproc.hh"
#include "bind_drivers.hh"
#include <pybind11/numpy.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <chrono>
#include <cstring>

namespace py = pybind11;
using namespace slate;

//------------------------------------------------------------------------------
// Host communicator implemented in Python.
class PyHostComm : public HostComm {
public:
    using HostComm::HostComm;
    int rank() const override { PYBIND11_OVERRIDE_PURE(int, HostComm, rank, ); }
    int size() const override { PYBIND11_OVERRIDE_PURE(int, HostComm, size, ); }
    std::string name() const override { return "python-host"; }
    void bcast_raw(void* buf, size_t count, ScalarType t, int root, hipStream_t) override {
        py::gil_scoped_acquire g;
        py::function f = py::get_override(static_cast<const HostComm*>(this), "bcast_raw");
        f(reinterpret_cast<uintptr_t>(buf), count * scalar_size(t), std::string(1, char(t)), root);
    }
    void allreduce_raw(const void* send, void* recv, size_t count, ScalarType t, ReduceOp op, hipStream_t) override {
        py::gil_scoped_acquire g;
        if (send != recv) std::memcpy(recv, send, count * scalar_size(t));
        py::function f = py::get_override(static_cast<const HostComm*>(this), "allreduce_raw");
        f(reinterpret_cast<uintptr_t>(recv), count, std::string(1, char(t)), std::string(1, char(op)));
    }
    void allgather_raw(const void* send, void* recv, size_t count, ScalarType t, hipStream_t) override {
        py::gil_scoped_acquire g;
        py::function f = py::get_override(static_cast<const HostComm*>(this), "allgather_raw");
        f(reinterpret_cast<uintptr_t>(send), reinterpret_cast<uintptr_t>(recv), count * scalar_size(t));
    }
    void send_raw(const void* buf, size_t count, ScalarType t, int peer, hipStream_t) override {
        py::gil_scoped_acquire g;
        py::function f = py::get_override(static_cast<const HostComm*>(this), "send_raw");
        f(reinterpret_cast<uintptr_t>(buf), count * scalar_size(t), peer);
    }
    void recv_raw(void* buf, size_t count, ScalarType t, int peer, hipStream_t) override {
        py::gil_scoped_acquire g;
        py::function f = py::get_override(static_cast<const HostComm*>(this), "recv_raw");
        f(reinterpret_cast<uintptr_t>(buf), count * scalar_size(t), peer);
    }
    void group_start() override {
        py::gil_scoped_acquire g;
        py::function f = py::get_override(static_cast<const HostComm*>(this), "group_start");
        if (f) f();
    }
    void group_end() override {
        py::gil_scoped_acquire g;
        py::function f = py::get_override(static_cast<const HostComm*>(this), "group_end");
        if (f) f();
    }
    void barrier() override {
        py::gil_scoped_acquire g;
        py::function f = py::get_override(static_cast<const HostComm*>(this), "barrier");
        f();
    }
};

//------------------------------------------------------------------------------
// DLPack (minimal ABI-compatible definitions)
namespace dl {
struct DLDevice { int32_t device_type; int32_t device_id; };
struct DLDataType { uint8_t code; uint8_t bits; uint16_t lanes; };
struct DLTensor { void* data; DLDevice device; int32_t ndim; DLDataType dtype; int64_t* shape; int64_t* strides; uint64_t byte_offset; };
struct DLManagedTensor { DLTensor dl_tensor; void* manager_ctx; void (*deleter)(DLManagedTensor*); };
constexpr int32_t kDLCPU = 1, kDLROCM = 10;
constexpr uint8_t kDLFloat = 2, kDLComplex = 5;

struct Ctx {
    std::shared_ptr<void> keep;
    int64_t shape[2];
    int64_t strides[2];
};

template <typename T>
DLDataType dtype_of() {
    if constexpr (std::is_same_v<T, float>) return {kDLFloat, 32, 1};
    else if constexpr (std::is_same_v<T, double>) return {kDLFloat, 64, 1};
    else if constexpr (std::is_same_v<T, std::complex<float>>) return {kDLComplex, 64, 1};
    else return {kDLComplex, 128, 1};
}

template <typename T>
py::capsule export_local(BaseMatrix<T> const& A, Loc loc) {
    LocalBlock<T> b = A.local(loc, false);
    auto* mt = new DLManagedTensor();
    auto* ctx = new Ctx();
    ctx->keep = A.storage();
    // column-major (m x n, ld) as a 2-D tensor with strides (1, ld)
    ctx->shape[0] = b.m; ctx->shape[1] = b.n;
    ctx->strides[0] = 1; ctx->strides[1] = b.ld;
    mt->dl_tensor.data = b.ptr ? static_cast<void*>(b.ptr) : reinterpret_cast<void*>(uintptr_t(256));
    mt->dl_tensor.device = {loc == Loc::Device ? kDLROCM : kDLCPU, loc == Loc::Device ? device::get_device() : 0};
    mt->dl_tensor.ndim = 2;
    mt->dl_tensor.dtype = dtype_of<T>();
    mt->dl_tensor.shape = ctx->shape;
    mt->dl_tensor.strides = ctx->strides;
    mt->dl_tensor.byte_offset = 0;
    mt->manager_ctx = ctx;
    mt->deleter = [](DLManagedTensor* self) {
        delete static_cast<Ctx*>(self->manager_ctx);
        delete self;
    };
    return py::capsule(mt, "dltensor", [](PyObject* cap) {
        if (PyCapsule_IsValid(cap, "dltensor")) {
            auto* m = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
            if (m && m->deleter) m->deleter(m);
        }
    });
}
}  // namespace dl

//------------------------------------------------------------------------------
Options to_options(py::dict d) {
    Options o;
    auto meth = [](py::handle v, Method (*parse)(std::string)) -> OptionValue {
        if (py::isinstance<py::str>(v)) return OptionValue(int64_t(parse(v.cast<std::string>())));
        return OptionValue(v.cast<int64_t>());
    };
    for (auto kv : d) {
        std::string k = py::str(kv.first);
        py::handle v = kv.second;
        if (k == "target") {
            if (py::isinstance<py::str>(v)) o[Option::Target] = str2target(v.cast<std::string>());
            else o[Option::Target] = v.cast<Target>();
        }
        else if (k == "lookahead") o[Option::Lookahead] = v.cast<int64_t>();
        else if (k == "block_size" || k == "nb") o[Option::BlockSize] = v.cast<int64_t>();
        else if (k == "inner_blocking" || k == "ib") o[Option::InnerBlocking] = v.cast<int64_t>();
        else if (k == "max_panel_threads") o[Option::MaxPanelThreads] = v.cast<int64_t>();
        else if (k == "tolerance") o[Option::Tolerance] = v.cast<double>();
        else if (k == "max_iterations") o[Option::MaxIterations] = v.cast<int64_t>();
        else if (k == "use_fallback_solver") o[Option::UseFallbackSolver] = v.cast<bool>();
        else if (k == "escalate_gmres") o[Option::EscalateGmres] = int64_t(v.cast<bool>());
        else if (k == "pivot_threshold") o[Option::PivotThreshold] = v.cast<double>();
        else if (k == "hold_local_workspace") o[Option::HoldLocalWorkspace] = v.cast<bool>();
        else if (k == "depth") o[Option::Depth] = v.cast<int64_t>();
        // methods: an int or the reference's names ("trsmA", "hemmC", "calu", ...)
        else if (k == "method_gemm") o[Option::MethodGemm] = meth(v, MethodGemm::str2method);
        else if (k == "method_lu") o[Option::MethodLU] = meth(v, MethodLU::str2method);
        else if (k == "method_trsm") o[Option::MethodTrsm] = meth(v, MethodTrsm::str2method);
        else if (k == "method_gels") o[Option::MethodGels] = meth(v, MethodGels::str2method);
        else if (k == "method_cholqr") o[Option::MethodCholQR] = meth(v, MethodCholQR::str2method);
        else if (k == "method_hemm") o[Option::MethodHemm] = meth(v, MethodHemm::str2method);
        else if (k == "method_eig") o[Option::MethodEig] = OptionValue(int64_t(v.cast<std::string>()[0]));
        else if (k == "print_verbose") o[Option::PrintVerbose] = v.cast<int64_t>();
        else if (k == "print_edge_items") o[Option::PrintEdgeItems] = v.cast<int64_t>();
        else if (k == "print_width") o[Option::PrintWidth] = v.cast<int64_t>();
        else if (k == "print_precision") o[Option::PrintPrecision] = v.cast<int64_t>();
        else throw Exception("unknown option: " + k);
    }
    return o;
}

//------------------------------------------------------------------------------
template <typename T>
void bind_type(py::module_& m, const char* sfx) {
    using R = real_type<T>;
    std::string s(sfx);
    auto BM = py::class_<BaseMatrix<T>>(m, ("BaseMatrix_" + s).c_str())
        .def_property_readonly("is_band_storage", [](BaseMatrix<T> const& A) { return A.storage()->banded; })
        .def_property_readonly("storage_bytes", [](BaseMatrix<T> const& A) {
            auto& st = *A.storage();
            return size_t(st.lld) * size_t(std::max<int64_t>(st.nloc, 1)) * sizeof(T);
        })
        .def_property_readonly("m", &BaseMatrix<T>::m)
        .def_property_readonly("n", &BaseMatrix<T>::n)
        .def_property_readonly("mt", &BaseMatrix<T>::mt)
        .def_property_readonly("nt", &BaseMatrix<T>::nt)
        .def_property_readonly("mb", &BaseMatrix<T>::mb)
        .def_property_readonly("nb", &BaseMatrix<T>::nb)
        .def_property_readonly("op", &BaseMatrix<T>::op)
        .def_property_readonly("uplo", &BaseMatrix<T>::uplo)
        .def_property_readonly("diag", &BaseMatrix<T>::diag)
        .def_property_readonly("kl", &BaseMatrix<T>::kl)
        .def_property_readonly("ku", &BaseMatrix<T>::ku)
        .def_property_readonly("grid", &BaseMatrix<T>::grid)
        .def("tileMb", &BaseMatrix<T>::tileMb)
        .def("tileNb", &BaseMatrix<T>::tileNb)
        .def("tileRank", &BaseMatrix<T>::tileRank)
        .def("tileIsLocal", &BaseMatrix<T>::tileIsLocal)
        // tile-level communication / layout (tile_comm.cc)
        .def("tileExists", &BaseMatrix<T>::tileExists)
        .def("tileLayout", &BaseMatrix<T>::tileLayout)
        .def("tileSend", &BaseMatrix<T>::tileSend, py::arg("i"), py::arg("j"), py::arg("dst_rank"), py::arg("tag") = 0)
        .def("tileRecv", &BaseMatrix<T>::tileRecv, py::arg("i"), py::arg("j"), py::arg("src_rank"),
             py::arg("layout") = Layout::ColMajor, py::arg("tag") = 0)
        .def("tileBcast", &BaseMatrix<T>::tileBcast, py::arg("i"), py::arg("j"), py::arg("B"),
             py::arg("layout") = Layout::ColMajor, py::arg("tag") = 0)
        .def("tileBcastToSet", &BaseMatrix<T>::tileBcastToSet, py::arg("i"), py::arg("j"), py::arg("ranks"),
             py::arg("layout") = Layout::ColMajor)
        .def("tileLayoutConvert", &BaseMatrix<T>::tileLayoutConvert)
        .def("tileLayoutReset", &BaseMatrix<T>::tileLayoutReset)
        .def("tileErase", &BaseMatrix<T>::tileErase)
        .def("tileData", [](BaseMatrix<T> const& A, int64_t i, int64_t j) {
            // logical tile (i, j) as a numpy array (host copy; layout and op applied)
            Loc loc = Loc::Host;
            if (!A.tileIsLocal(i, j)) {
                try { (void)A.tile(i, j, Loc::Host); } catch (...) { loc = Loc::Device; }
            } else {
                A.tileGetAllForReading(Loc::Host);
            }
            Tile<T> t = A.tile(i, j, loc);
            std::vector<T> h;
            if (loc == Loc::Device) {
                const int64_t rows = t.layout == Layout::ColMajor ? t.mb : t.nb;
                const int64_t cols = t.layout == Layout::ColMajor ? t.nb : t.mb;
                h.resize(size_t(std::max<int64_t>(rows * cols, 1)));
                slate_hip_call(hipMemcpy2D(h.data(), rows * sizeof(T), t.data, t.stride * sizeof(T), rows * sizeof(T),
                                           cols, hipMemcpyDeviceToHost));
                t.data = h.data();
                t.stride = std::max<int64_t>(rows, 1);
            }
            py::array_t<T, py::array::f_style> out({t.mb_(), t.nb_()});
            auto r = out.template mutable_unchecked<2>();
            for (int64_t jj = 0; jj < t.nb_(); ++jj)
                for (int64_t ii = 0; ii < t.mb_(); ++ii) r(ii, jj) = t.at(ii, jj);
            return out;
        })
        .def("mpiRank", &BaseMatrix<T>::mpiRank)
        .def("local_shape", [](BaseMatrix<T> const& A) {
            return py::make_tuple(A.lrow_end() - A.lrow_begin(), A.lcol_end() - A.lcol_begin());
        })
        .def("local_row_indices", [](BaseMatrix<T> const& A) {
            // global (view-relative, storage orientation) row index of each local row
            auto& st = *A.storage();
            std::vector<int64_t> r;
            for (int64_t l = A.lrow_begin(); l < A.lrow_end(); ++l)
                r.push_back(l2g(l, st.mb, st.rrel(), st.grid->p()) - A.row0());
            return r;
        })
        .def("local_col_indices", [](BaseMatrix<T> const& A) {
            auto& st = *A.storage();
            std::vector<int64_t> r;
            for (int64_t l = A.lcol_begin(); l < A.lcol_end(); ++l)
                r.push_back(l2g(l, st.nb, st.crel(), st.grid->q()) - A.col0());
            return r;
        })
        .def("get_local", [](BaseMatrix<T> const& A) {
            // copy of the local block (storage orientation) as Fortran-order numpy
            LocalBlock<T> b = A.local(Loc::Host, false);
            py::array_t<T, py::array::f_style> out({b.m, b.n});
            T* o = out.mutable_data();
            for (int64_t j = 0; j < b.n; ++j)
                if (b.m) std::memcpy(o + j * b.m, b.ptr + j * b.ld, b.m * sizeof(T));
            return out;
        })
        .def("set_local", [](BaseMatrix<T>& A, py::array_t<T, py::array::f_style | py::array::forcecast> a) {
            LocalBlock<T> b = A.local(Loc::Host, true);
            if (a.ndim() != 2 || a.shape(0) != b.m || a.shape(1) != b.n)
                throw Exception("set_local: shape mismatch");
            const T* src = a.data();
            for (int64_t j = 0; j < b.n; ++j)
                if (b.m) std::memcpy(b.ptr + j * b.ld, src + j * b.m, b.m * sizeof(T));
        })
        .def("local_dlpack", [](BaseMatrix<T> const& A, bool device) {
            return dl::export_local<T>(A, device ? Loc::Device : Loc::Host);
        }, py::arg("device") = true)
        .def("mark_modified", [](BaseMatrix<T>& A, bool device) {
            A.storage()->modified(device ? Loc::Device : Loc::Host);
        }, py::arg("device") = true)
        .def("gather", [](BaseMatrix<T> const& A) {
            std::vector<T> full;
            {
                py::gil_scoped_release r;
                gather(A, full);
            }
            py::array_t<T, py::array::f_style> out({A.m(), A.n()});
            if (!full.empty()) std::memcpy(out.mutable_data(), full.data(), full.size() * sizeof(T));
            return out;
        })
        .def("insertLocalTiles", [](BaseMatrix<T>& A, Target t) {
            Matrix<T>(A).insertLocalTiles(t);
        }, py::arg("target") = Target::Host)
        .def("tileUpdateAllOrigin", &BaseMatrix<T>::tileUpdateAllOrigin)
        .def("releaseWorkspace", &BaseMatrix<T>::releaseWorkspace)
        .def("origin_is_device", [](BaseMatrix<T> const& A) { return A.storage()->origin() == Loc::Device; })
        .def_property_readonly("is_multi_device", &BaseMatrix<T>::is_multi_device)
        .def_property_readonly("num_parts", [](BaseMatrix<T> const& A) {
            return A.is_multi_device() ? int(A.storage()->parts.size()) : 1;
        });

    py::class_<Matrix<T>, BaseMatrix<T>>(m, ("Matrix_" + s).c_str())
        .def(py::init([](int64_t mm, int64_t n, int64_t mb, int64_t nb, GridPtr g) {
            return Matrix<T>(mm, n, mb, nb, g ? g : default_grid());
        }), py::arg("m"), py::arg("n"), py::arg("mb"), py::arg("nb"), py::arg("grid") = nullptr)
        .def(py::init([](BaseMatrix<T> const& b) { return Matrix<T>(b); }))
        // arbitrary distribution (reference lambda constructor): tile row /
        // column sizes and the owning world rank of every tile (mt x nt list)
        .def_static("with_layout", [](int64_t mm, int64_t n, std::vector<int64_t> rsz, std::vector<int64_t> csz,
                                      std::vector<std::vector<int>> owner, GridPtr g) {
            auto tmb = [rsz](int64_t i) { return i < int64_t(rsz.size()) ? rsz[i] : rsz.back(); };
            auto tnb = [csz](int64_t j) { return j < int64_t(csz.size()) ? csz[j] : csz.back(); };
            auto trk = [owner](std::tuple<int64_t, int64_t> ij) {
                return owner.at(std::get<0>(ij)).at(std::get<1>(ij));
            };
            auto tdv = [](std::tuple<int64_t, int64_t>) { return 0; };
            return Matrix<T>(mm, n, tmb, tnb, trk, tdv, g ? g : default_grid());
        }, py::arg("m"), py::arg("n"), py::arg("row_sizes"), py::arg("col_sizes"), py::arg("owner"),
           py::arg("grid") = nullptr)
        .def("arbitrary_layout", &BaseMatrix<T>::arbitrary_layout)
        // multi-device matrices (reference fromDevices(Aarray, num_devices)):
        // 2-D block-cyclic over num_devices in-process ranks, or the
        // reference's 1-D tile-column layout over given per-device arrays
        .def_static("multiDevice", [](int64_t mm, int64_t n, int64_t mb, int64_t nb, int num_devices) {
            py::gil_scoped_release r;
            return Matrix<T>::multiDevice(mm, n, mb, nb, num_devices);
        }, py::arg("m"), py::arg("n"), py::arg("mb"), py::arg("nb"), py::arg("num_devices") = 0)
        .def_static("fromDevicesArray", [](int64_t mm, int64_t n, std::vector<uintptr_t> ptrs, int64_t lda,
                                           int64_t mb, int64_t nb) {
            std::vector<T*> a;
            for (auto p : ptrs) a.push_back(reinterpret_cast<T*>(p));
            return Matrix<T>::fromDevices(mm, n, a.data(), int(a.size()), lda, mb, nb);
        })
        .def("gather_into", [](Matrix<T> const& A, py::array_t<T, py::array::f_style> out) {
            py::buffer_info bi = out.request();
            slate_error_if_msg(bi.ndim != 2 || bi.shape[0] < A.m() || bi.shape[1] < A.n(), "gather_into: shape");
            T* ptr = static_cast<T*>(bi.ptr);
            const int64_t ld = bi.shape[0];
            py::gil_scoped_release r;
            A.gather(ptr, ld);
        })
        .def_static("fromDevicePointer", [](int64_t mm, int64_t n, uintptr_t ptr, int64_t lld, int64_t mb,
                                              int64_t nb, GridPtr g) {
            return Matrix<T>::fromScaLAPACK(mm, n, reinterpret_cast<T*>(ptr), lld, mb, nb, g, Loc::Device);
        })
        .def_static("fromHostPointer", [](int64_t mm, int64_t n, uintptr_t ptr, int64_t lld, int64_t mb,
                                            int64_t nb, GridPtr g) {
            return Matrix<T>::fromScaLAPACK(mm, n, reinterpret_cast<T*>(ptr), lld, mb, nb, g, Loc::Host);
        })
        .def("sub", &Matrix<T>::sub)
        .def("slice", &Matrix<T>::slice)
        .def("emptyLike", &Matrix<T>::emptyLike, py::arg("mb") = 0, py::arg("nb") = 0, py::arg("deepOp") = Op::NoTrans)
        .def("transpose", [](Matrix<T> const& A) { return transpose(A); })
        .def("conj_transpose", [](Matrix<T> const& A) { return conj_transpose(A); });

    py::class_<BaseTrapezoidMatrix<T>, BaseMatrix<T>>(m, ("BaseTrapezoidMatrix_" + s).c_str());
    py::class_<TrapezoidMatrix<T>, BaseTrapezoidMatrix<T>>(m, ("TrapezoidMatrix_" + s).c_str())
        .def(py::init<Uplo, Diag, BaseMatrix<T> const&>())
        .def("transpose", [](TrapezoidMatrix<T> const& A) { return transpose(A); })
        .def("conj_transpose", [](TrapezoidMatrix<T> const& A) { return conj_transpose(A); });
    py::class_<TriangularMatrix<T>, BaseTrapezoidMatrix<T>>(m, ("TriangularMatrix_" + s).c_str())
        .def(py::init<Uplo, Diag, BaseMatrix<T> const&>())
        .def("transpose", [](TriangularMatrix<T> const& A) { return transpose(A); })
        .def("conj_transpose", [](TriangularMatrix<T> const& A) { return conj_transpose(A); });
    py::class_<SymmetricMatrix<T>, BaseTrapezoidMatrix<T>>(m, ("SymmetricMatrix_" + s).c_str())
        .def(py::init<Uplo, BaseMatrix<T> const&>())
        .def("transpose", [](SymmetricMatrix<T> const& A) { return transpose(A); });
    py::class_<HermitianMatrix<T>, BaseTrapezoidMatrix<T>>(m, ("HermitianMatrix_" + s).c_str())
        .def(py::init<Uplo, BaseMatrix<T> const&>())
        .def("conj_transpose", [](HermitianMatrix<T> const& A) { return conj_transpose(A); });
    py::class_<BandMatrix<T>, BaseMatrix<T>>(m, ("BandMatrix_" + s).c_str())
        .def(py::init<int64_t, int64_t, BaseMatrix<T> const&>())
        // band-only storage (reference BandMatrix(m, n, kl, ku, nb, ...) ctor)
        .def_static("banded", [](int64_t mm, int64_t n, int64_t kl, int64_t ku, int64_t nb, GridPtr g) {
            return BandMatrix<T>(mm, n, kl, ku, nb, g ? g : default_grid());
        }, py::arg("m"), py::arg("n"), py::arg("kl"), py::arg("ku"), py::arg("nb"), py::arg("grid") = nullptr)
        .def("transpose", [](BandMatrix<T> const& A) { return transpose(A); })
        .def("conj_transpose", [](BandMatrix<T> const& A) { return conj_transpose(A); });
    py::class_<TriangularBandMatrix<T>, BaseMatrix<T>>(m, ("TriangularBandMatrix_" + s).c_str())
        .def(py::init<Uplo, Diag, int64_t, BaseMatrix<T> const&>())
        .def_static("banded", [](Uplo u, Diag d, int64_t n, int64_t kd, int64_t nb, GridPtr g) {
            return TriangularBandMatrix<T>(u, d, n, kd, nb, g ? g : default_grid());
        }, py::arg("uplo"), py::arg("diag"), py::arg("n"), py::arg("kd"), py::arg("nb"), py::arg("grid") = nullptr)
        .def("transpose", [](TriangularBandMatrix<T> const& A) { return transpose(A); })
        .def("conj_transpose", [](TriangularBandMatrix<T> const& A) { return conj_transpose(A); });
    py::class_<HermitianBandMatrix<T>, BaseMatrix<T>>(m, ("HermitianBandMatrix_" + s).c_str())
        .def(py::init<Uplo, int64_t, BaseMatrix<T> const&>())
        .def_static("banded", [](Uplo u, int64_t n, int64_t kd, int64_t nb, GridPtr g) {
            return HermitianBandMatrix<T>(u, n, kd, nb, g ? g : default_grid());
        }, py::arg("uplo"), py::arg("n"), py::arg("kd"), py::arg("nb"), py::arg("grid") = nullptr);

    bind_drivers<T>(m, s);
}

PYBIND11_MODULE(_slate, m) {
    m.doc() = "slate_d35_amd native library (MI355X / gfx950)";

    py::enum_<Target>(m, "Target")
        .value("Host", Target::Host).value("HostTask", Target::HostTask).value("HostNest", Target::HostNest)
        .value("HostBatch", Target::HostBatch).value("Devices", Target::Devices);
    py::enum_<Op>(m, "Op").value("NoTrans", Op::NoTrans).value("Trans", Op::Trans).value("ConjTrans", Op::ConjTrans);
    py::enum_<Uplo>(m, "Uplo").value("Upper", Uplo::Upper).value("Lower", Uplo::Lower).value("General", Uplo::General);
    py::enum_<Diag>(m, "Diag").value("NonUnit", Diag::NonUnit).value("Unit", Diag::Unit);
    py::enum_<Side>(m, "Side").value("Left", Side::Left).value("Right", Side::Right);
    py::enum_<Norm>(m, "Norm").value("One", Norm::One).value("Two", Norm::Two).value("Inf", Norm::Inf)
        .value("Fro", Norm::Fro).value("Max", Norm::Max);
    py::enum_<Layout>(m, "Layout").value("ColMajor", Layout::ColMajor).value("RowMajor", Layout::RowMajor);
    py::enum_<GridOrder>(m, "GridOrder").value("Col", GridOrder::Col).value("Row", GridOrder::Row);
    py::enum_<Equed>(m, "Equed").value("None_", Equed::None).value("Row", Equed::Row).value("Col", Equed::Col)
        .value("Both", Equed::Both);
    py::enum_<Job>(m, "Job").value("NoVec", Job::NoVec).value("Vec", Job::Vec);

    py::class_<Comm, std::shared_ptr<Comm>>(m, "Comm")
        .def("rank", &Comm::rank)
        .def("size", &Comm::size)
        .def("name", &Comm::name)
        .def("device", &Comm::device)
        .def("barrier", &Comm::barrier, py::call_guard<py::gil_scoped_release>())
        .def("allreduce_sum_i64", [](Comm& c, std::vector<int64_t> v) {
            if (!v.empty()) c.allreduce(v.data(), v.data(), v.size(), ScalarType::Int64, ReduceOp::Sum, Loc::Host, nullptr);
            return v;
        }, py::call_guard<py::gil_scoped_release>());
    py::class_<SelfComm, Comm, std::shared_ptr<SelfComm>>(m, "SelfComm").def(py::init<>());
    py::class_<HostComm, PyHostComm, Comm, std::shared_ptr<HostComm>>(m, "HostComm").def(py::init<>());
    m.def("lu_rowx_stats", []() { int64_t e = 0, r = 0; lu_rowx_stats(e, r); return py::make_tuple(e, r); });
    m.def("lu_rowx_reset", &lu_rowx_reset);
    m.def("inproc_run_count", &inproc_run_count);
    // self-check of the in-process all-reduce (small: all-to-all copies;
    // >= 1 MiB with > 2 ranks: reduce-scatter + all-gather): every rank
    // contributes x_r[i] = r + i * 1e-3; returns the max error over ranks
    // rounds > 1: every round is a (large) all-reduce immediately followed by
    // a bcast and a small all-reduce, with rank-dependent host delays, so a
    // fast rank enters the next collective while a slow one is still in the
    // last hand-off of the previous one (sliced all-reduce phase 3)
    m.def("inproc_allreduce_check", [](int nranks, int64_t count, int rounds) {
        std::vector<double> err(nranks, 0.0);
        {
            py::gil_scoped_release r;
            run_in_process(1, nranks, [&](int rank, GridPtr const& g) {
                const bool dev = device::available();
                const Loc loc = dev ? Loc::Device : Loc::Host;
                std::vector<double> h(count), hs(64);
                device::Buffer<double> d(dev ? count : 0), ds(dev ? 64 : 0);
                hipStream_t st = dev ? device::queue(0) : nullptr;
                double* p = dev ? d.data() : h.data();
                double* ps = dev ? ds.data() : hs.data();
                double e = 0;
                for (int it = 0; it < rounds; ++it) {
                    for (int64_t i = 0; i < count; ++i) h[i] = rank + it + double(i % 1000) * 1e-3;
                    for (int i = 0; i < 64; ++i) hs[i] = rank == it % nranks ? double(it * 100 + i) : -1.0;
                    if (dev) {
                        device::memcpy_async(d.data(), h.data(), count * 8, st);
                        device::memcpy_async(ds.data(), hs.data(), 64 * 8, st);
                    }
                    if ((rank + it) % nranks == 0) std::this_thread::sleep_for(std::chrono::milliseconds(2));
                    g->world().allreduce(p, p, size_t(count), ScalarType::Float64, ReduceOp::Sum, loc, st);
                    if ((rank + it) % nranks == 1) std::this_thread::sleep_for(std::chrono::milliseconds(2));
                    g->world().bcast(ps, 64, ScalarType::Float64, it % nranks, loc, st);
                    g->world().allreduce(ps, ps, 64, ScalarType::Float64, ReduceOp::Max, loc, st);
                    if (dev) {
                        device::memcpy_async(h.data(), d.data(), count * 8, st);
                        device::memcpy_async(hs.data(), ds.data(), 64 * 8, st);
                        slate_hip_call(hipStreamSynchronize(st));
                    }
                    const double base = nranks * (nranks - 1) / 2.0 + double(nranks) * it;
                    for (int64_t i = 0; i < count; ++i)
                        e = std::max(e, std::abs(h[i] - (base + nranks * double(i % 1000) * 1e-3)));
                    for (int i = 0; i < 64; ++i) e = std::max(e, std::abs(hs[i] - double(it * 100 + i)));
                }
                err[rank] = e;
            });
        }
        return *std::max_element(err.begin(), err.end());
    }, py::arg("nranks"), py::arg("count"), py::arg("rounds") = 1);
    m.def("inproc_copy_bytes", &inproc_copy_bytes);
    m.def("inproc_last_shape", []() { int p = 0, q = 0; inproc_last_shape(p, q); return py::make_tuple(p, q); });
    m.def("comm_abort_all", &comm_abort_all, py::call_guard<py::gil_scoped_release>());
    m.def("comm_async_errors", &comm_async_errors);
    m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });
    m.def("make_rccl_comm", [](py::bytes uid, int nranks, int rank) {
        std::string s = uid;
        py::gil_scoped_release r;
        return make_rccl_comm(s, nranks, rank);
    });
    m.def("rccl_split", [](CommPtr parent, int color, int key) {
        py::gil_scoped_release r;
        return rccl_split(parent, color, key);
    });

    // native bootstrap + TCP host transport (csrc/src/tcp_comm.cc)
    m.def("make_tcp_world", [](double timeout) { return make_tcp_world(timeout); },
          py::arg("timeout") = 120.0, py::call_guard<py::gil_scoped_release>());
    m.def("tcp_split", [](CommPtr parent, int color, int key) { return tcp_split(parent, color, key); },
          py::call_guard<py::gil_scoped_release>());
    m.def("native_init_grid", [](int p, int q, GridOrder order, std::string transport) {
        return slate::init_grid(p, q, order, transport); },
          py::arg("p") = 0, py::arg("q") = 0, py::arg("order") = GridOrder::Col, py::arg("transport") = "auto",
          py::call_guard<py::gil_scoped_release>());
    m.def("native_finalize", &slate::finalize, py::call_guard<py::gil_scoped_release>());
    py::class_<Grid, std::shared_ptr<Grid>>(m, "Grid")
        .def(py::init<int, int, GridOrder, CommPtr, CommPtr, CommPtr>())
        .def_static("self", &Grid::self)
        .def_property_readonly("p", &Grid::p)
        .def_property_readonly("q", &Grid::q)
        .def_property_readonly("order", &Grid::order)
        .def_property_readonly("rank", &Grid::rank)
        .def_property_readonly("myrow", &Grid::myrow)
        .def_property_readonly("mycol", &Grid::mycol)
        .def("rank_of", &Grid::rank_of)
        .def("transposed", &Grid::transposed)
        .def_property_readonly("world", &Grid::world_ptr)
        .def_property_readonly("row_comm", &Grid::row_ptr)
        .def_property_readonly("col_comm", &Grid::col_ptr)
        .def("set_fast", &Grid::set_fast)
        .def_property_readonly("has_fast_lane", &Grid::has_fast_lane);
    m.def("generate_matrix_usage", &slate::generate_matrix_usage);
    m.def("default_grid", &default_grid);
    m.def("set_default_grid", &set_default_grid);

    // device runtime
    m.def("device_available", &device::available);
    m.def("device_count", &device::count);
    m.def("set_device", &device::set_device);
    m.def("get_device", &device::get_device);
    m.def("sync", &slate::sync, py::call_guard<py::gil_scoped_release>());
    m.def("set_ops_queue", [](int q) { ops_queue() = q; });
    m.def("queue_sync", [](int q) { slate_hip_call(hipStreamSynchronize(device::queue(q))); },
          py::call_guard<py::gil_scoped_release>());
    m.def("release_cache", &device::release_cache);
    m.def("lane_log_enable", &Sched::lane_log_enable);
    m.def("storage_alloc_max", &storage_alloc_max);
    m.def("storage_alloc_reset", &storage_alloc_reset);
    m.def("lane_log_take", &Sched::lane_log_take);
    m.def("bytes_in_use", &device::bytes_in_use);
    m.def("debug_on", &Debug::on);
    m.def("debug_off", &Debug::off);
    m.def("debug_enabled", &Debug::enabled);
    m.def("debug_mem_report", &Debug::printNumFreeMemBlocks);
    m.def("debug_device_leaks", &Debug::checkDeviceMemoryLeaks);
    m.def("debug_host_leaks", &Debug::checkHostMemoryLeaks);
    m.def("version", &slate::version);
    // tridiagonal / bidiagonal host solvers (fp64): return numpy arrays
    using VD = std::vector<double>;
    auto mat = [](std::vector<double> const& v, int64_t r, int64_t c) {
        py::array_t<double, py::array::f_style> a({r, c});
        std::copy(v.begin(), v.end(), a.mutable_data());
        return a;
    };
    m.def("sterf", [](VD d, VD e) { slate::host::sterf<double>(int64_t(d.size()), d.data(), e.data()); return d; });
    m.def("steqr", [=](VD d, VD e, bool vectors) {
        int64_t n = d.size();
        VD Z(vectors ? n * n : 0);
        for (int64_t i = 0; vectors && i < n; ++i) Z[i + i * n] = 1;
        slate::host::steqr<double, double>(n, d.data(), e.data(), vectors ? Z.data() : nullptr, n, vectors ? n : 0);
        return py::make_tuple(d, mat(Z, vectors ? n : 0, vectors ? n : 0)); });
    m.def("stedc", [=](VD d, VD e) {
        int64_t n = d.size();
        VD Z(n * n);
        slate::host::stedc<double>(n, d.data(), e.data(), Z.data(), n);
        return py::make_tuple(d, mat(Z, n, n)); });
    m.def("bdsqr", [=](VD d, VD e) {
        int64_t n = d.size();
        VD U(n * n), VT(n * n);
        for (int64_t i = 0; i < n; ++i) { U[i + i * n] = 1; VT[i + i * n] = 1; }
        slate::host::bdsqr<double, double>(n, d.data(), e.data(), U.data(), n, n, VT.data(), n, n);
        return py::make_tuple(d, mat(U, n, n), mat(VT, n, n)); });
    // bdsqr's host loop alone (rotations generated and handed to a sink that
    // only keeps them, as the device sink's batching does): its cost bounds
    // the device SVD's bdsqr stage
    m.def("bdsqr_core_bench", [](VD d, VD e) {
        struct KeepSink : slate::host::RotSink<double> {
            std::vector<std::vector<slate::host::PlaneRot<double>>> keep_u, keep_v;
            size_t count = 0;
            void sweep(std::vector<slate::host::PlaneRot<double>>& ru,
                       std::vector<slate::host::PlaneRot<double>>& rv) override {
                count += ru.size() + rv.size();
                keep_u.emplace_back(); keep_u.back().swap(ru);
                keep_v.emplace_back(); keep_v.back().swap(rv);
                if (keep_u.size() == 16) { keep_u.clear(); keep_v.clear(); }
            }
            void rot_u(int64_t, int64_t, double, double) override {}
            void negate_v(int64_t) override {}
            void permute(std::vector<int64_t> const&) override {}
        } sink;
        const int64_t n = d.size();
        auto t0 = std::chrono::steady_clock::now();
        slate::host::bdsqr_core<double>(n, d.data(), e.data(), &sink);
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return py::make_tuple(d, dt, sink.count); });
    m.def("timers", []() { return timers(); });
    m.def("clear_timers", []() { timers().clear(); });

    // tracing
    auto tr = m.def_submodule("trace");
    tr.def("on", &trace::Trace::on);
    tr.def("off", &trace::Trace::off);
    tr.def("is_on", &trace::Trace::is_on);
    tr.def("comment", &trace::Trace::comment);
    tr.def("clear", &trace::Trace::clear);
    tr.def("finish", [](CommPtr c, std::string base) {
        py::gil_scoped_release r;
        return trace::Trace::finish(c.get(), base);
    }, py::arg("comm") = nullptr, py::arg("basename") = "");
    tr.def("events", []() {
        py::list out;
        for (auto& e : trace::Trace::events())
            out.append(py::make_tuple(std::string(e.name), e.start, e.stop, e.lane));
        return out;
    });

    m.def("options", &to_options);

    bind_type<float>(m, "s");
    bind_type<double>(m, "d");
    bind_type<std::complex<float>>(m, "c");
    bind_type<std::complex<double>>(m, "z");
    bind_mixed(m);
}
