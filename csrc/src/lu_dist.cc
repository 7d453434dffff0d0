// Host / device dispatch of the distributed LU row-permutation helpers
// (device kernels: kernels/lu_dist.hip; see there for the slot scheme).
#include "lu_dist.hh"

#include <cstring>
#include <cstdlib>
#include <functional>
#include <vector>

namespace slate {
namespace internal {
namespace ludist {

namespace kd = slate_amd::dev;
using kd::dptr;

template <typename T>
void gather_rows_ids(lb::Ctx const& c, int64_t cnt, int64_t ncols, int64_t const* sel, T const* A, int64_t lda,
                     T* out, int64_t ldo, int64_t const* id_in, int64_t* id_out, RowDist const& d, int64_t li_base) {
    if (cnt <= 0) return;
    if (c.dev()) {
        kd::gather_rows_ids(cnt, ncols, sel, dptr(A), lda, dptr(out), ldo, id_in, id_out, d, li_base, c.stream);
        return;
    }
    for (int64_t i = 0; i < cnt; ++i) {
        if (id_out) id_out[i] = id_in ? id_in[sel[i]] : kd::rd_l2g(d, li_base + sel[i]);
        for (int64_t j = 0; j < ncols; ++j) out[i + j * ldo] = A[sel[i] + j * lda];
    }
}

void perm_slots(lb::Ctx const& c, int mode, int64_t base, int cnt, int64_t const* in, int64_t in_off,
                int64_t* ipiv_out, int64_t* slot_src, int64_t* slot_dst) {
    if (cnt <= 0) return;
    slate_error_if_msg(cnt > 1024, "distributed LU: tile size above 1024");
    if (c.dev()) {
        kd::perm_slots(mode, base, cnt, in, in_off, ipiv_out, slot_src, slot_dst, c.stream);
        return;
    }
    // same replay as the kernel (slot table: pos[s], content[s])
    std::vector<int64_t> pos(2 * cnt);
    std::vector<int> content(2 * cnt);
    int n = cnt;
    for (int s = 0; s < cnt; ++s) { pos[s] = base + s; content[s] = s; }
    for (int t = 0; t < cnt; ++t) {
        int64_t key = in[t] + in_off;
        int f = -1;
        for (int s = 0; s < n && f < 0; ++s)
            if (mode == 0 ? pos[content[s]] == key : pos[s] == key) f = s;
        if (f < 0) { f = n++; pos[f] = key; content[f] = f; }
        ipiv_out[t] = pos[f];
        std::swap(content[t], content[f]);
    }
    for (int s = 0; s < 2 * cnt; ++s) {
        slot_src[s] = s < n ? pos[content[s]] : -1;
        slot_dst[s] = s < n ? pos[s] : -1;
    }
}

template <typename T>
void slots_pack(lb::Ctx const& c, int s0, int s1, int64_t ncols, int64_t const* slot_src, T const* A, int64_t lda,
                RowDist const& d, T* buf, int64_t ldb) {
    if (s1 <= s0 || ncols <= 0) return;
    if (c.dev()) {
        kd::slots_pack(s0, s1, ncols, slot_src, dptr(A), lda, d, dptr(buf), ldb, c.stream);
        return;
    }
    for (int s = s0; s < s1; ++s) {
        int64_t src = slot_src[s];
        bool mine = src >= 0 && kd::rd_owner(d, src) == d.myrow;
        int64_t lr = mine ? kd::rd_lrow(d, src) : 0;
        for (int64_t j = 0; j < ncols; ++j) buf[(s - s0) + j * ldb] = mine ? A[lr + j * lda] : T(0);
    }
}

template <typename T>
void slots_unpack(lb::Ctx const& c, int s0, int s1, int64_t ncols, int64_t const* slot_dst, T const* buf,
                  int64_t ldb, T* A, int64_t lda, RowDist const& d) {
    if (s1 <= s0 || ncols <= 0) return;
    if (c.dev()) {
        kd::slots_unpack(s0, s1, ncols, slot_dst, dptr(buf), ldb, dptr(A), lda, d, c.stream);
        return;
    }
    for (int s = s0; s < s1; ++s) {
        int64_t dst = slot_dst[s];
        if (dst < 0 || kd::rd_owner(d, dst) != d.myrow) continue;
        int64_t lr = kd::rd_lrow(d, dst);
        for (int64_t j = 0; j < ncols; ++j) A[lr + j * lda] = buf[(s - s0) + j * ldb];
    }
}

namespace {
template <typename T> T unit_phase(T b) {
    if constexpr (is_complex_v<T>) {
        return T(std::real(b) < 0 ? -1 : 1);   // real +-1: R keeps a real diagonal (tsqr.hip)
    } else {
        return b < T(0) ? T(-1) : T(1);
    }
}
}  // namespace

template <typename T>
void lu_sign(lb::Ctx const& c, int64_t n, T* A, int64_t lda, T* sgn) {
    if (n <= 0) return;
    if (!c.dev()) {
        for (int64_t k = 0; k < n; ++k) {
            T s = unit_phase(A[k + k * lda]);
            A[k + k * lda] += s;
            sgn[k] = s;
            T d = A[k + k * lda];
            for (int64_t i = k + 1; i < n; ++i) A[i + k * lda] /= d;
            for (int64_t j = k + 1; j < n; ++j) {
                T u = A[k + j * lda];
                for (int64_t i = k + 1; i < n; ++i) A[i + j * lda] -= A[i + k * lda] * u;
            }
        }
        return;
    }
    // 64-column leaves (tsqr.hip lu_sign_leaf: diagonal block, L21 and U12
    // in one launch) and one GEMM per leaf; SLATE_LU_SIGN_LEAF=0 keeps the
    // recursion over 32-column narrow blocks
    static const bool leaf = [] {
        const char* e = std::getenv("SLATE_LU_SIGN_LEAF");
        return e ? std::atoi(e) != 0 : true;
    }();
    if (sizeof(T) <= 8 && leaf) {
        lb::Scratch sc(c);
        T* Wk[2] = {sc.alloc<T>(64 * 64), sc.alloc<T>(64 * 64)};
        T* Aprev = nullptr;
        int bprev = 0;
        for (int64_t c0 = 0, k = 0; c0 < n; c0 += 64, ++k) {
            const int64_t b = std::min<int64_t>(64, n - c0), r = n - c0 - b;
            kd::lu_sign_leaf<kd::dev_t<T>>(n, c0, int(b), dptr(A), lda, dptr(sgn), dptr(Wk[k & 1]),
                                           Aprev ? dptr(Wk[(k + 1) & 1]) : nullptr, dptr(Aprev), bprev, c.stream);
            Aprev = A + c0 + c0 * lda;
            bprev = int(b);
            if (r == 0) break;
            lb::gemm(c, Op::NoTrans, Op::NoTrans, r, r, b, T(-1), A + (c0 + b) + c0 * lda, lda,
                     A + c0 + (c0 + b) * lda, lda, T(1), A + (c0 + b) + (c0 + b) * lda, lda);
        }
        return;
    }
    // right-looking recursion over 32-column narrow blocks (tsqr.hip)
    lb::Scratch sc(c);
    T* Utop = sc.alloc<T>(32 * 32);
    std::function<void(int64_t, int64_t)> rec = [&](int64_t c0, int64_t nn) {
        if (nn <= 32) {
            lb::copy2d(c, nn, nn, A + c0 + c0 * lda, lda, Utop, int64_t(32));
            kd::lu_sign_narrow(n, c0, int(nn), dptr(A), lda, dptr(Utop), dptr(sgn), c.stream);
            return;
        }
        int64_t n1 = ((nn + 1) / 2 + 31) / 32 * 32, n2 = nn - n1;
        rec(c0, n1);
        lb::trsm(c, Side::Left, Uplo::Lower, Op::NoTrans, Diag::Unit, n1, n2, T(1), A + c0 + c0 * lda, lda,
                 A + c0 + (c0 + n1) * lda, lda);
        lb::gemm(c, Op::NoTrans, Op::NoTrans, n - c0 - n1, n2, n1, T(-1), A + (c0 + n1) + c0 * lda, lda,
                 A + c0 + (c0 + n1) * lda, lda, T(1), A + (c0 + n1) + (c0 + n1) * lda, lda);
        rec(c0 + n1, n2);
    };
    rec(0, n);
}

template <typename T>
int64_t pplu_entry(int64_t kb) { return kd::pplu_entry<kd::dev_t<T>>(kb); }

namespace {
template <typename T>
inline int64_t pp_hdr(int64_t kb) { return pplu_entry<T>(kb) - 2 * kb; }
template <typename T>
inline real_type<T>& pp_val(T* e) { return *reinterpret_cast<real_type<T>*>(e); }
template <typename T>
inline int64_t& pp_gid(T* e) { return *reinterpret_cast<int64_t*>(reinterpret_cast<char*>(e) + 8); }
}  // namespace

template <typename T>
void pplu_cand(lb::Ctx const& c, int64_t mr, int64_t j, int64_t r0, T const* ap, int64_t lda, int64_t kb,
               RowDist const& d, int64_t lr_k, bool is_pk, T* buf) {
    if (c.dev()) {
        kd::pplu_cand(mr, j, r0, dptr(ap), lda, kb, d, lr_k, is_pk, dptr(buf), c.stream);
        return;
    }
    using R = real_type<T>;
    R best = R(-1);
    int64_t bi = -1;
    for (int64_t r = r0; r < mr; ++r) {
        R v = std::abs(std::real(ap[r + j * lda])) + std::abs(std::imag(ap[r + j * lda]));
        if (v > best) { best = v; bi = r; }
    }
    const int64_t hdr = pp_hdr<T>(kb);
    std::fill(buf, buf + hdr, T(0));
    pp_val(buf) = best;
    pp_gid(buf) = bi >= 0 ? kd::rd_l2g(d, lr_k + bi) : -1;
    for (int64_t cc = 0; cc < kb; ++cc) {
        buf[hdr + cc] = bi >= 0 ? ap[bi + cc * lda] : T(0);
        buf[hdr + kb + cc] = is_pk ? ap[j + cc * lda] : T(0);
    }
}

template <typename T>
void pplu_apply(lb::Ctx const& c, int np, T const* gbuf, int64_t kb, int64_t j, int64_t cend, int64_t mr,
                int64_t r_upd0, T* ap, int64_t lda, RowDist const& d, int64_t lr_k, int64_t kk, int pk, double thresh,
                bool is_pk, int64_t* pip, int* info, int64_t info_off) {
    if (c.dev()) {
        kd::pplu_apply(np, dptr(gbuf), kb, j, cend, mr, r_upd0, dptr(ap), lda, d, lr_k, kk, pk, thresh, is_pk, pip,
                       info, info_off, c.stream);
        return;
    }
    using R = real_type<T>;
    const int64_t E = pplu_entry<T>(kb), hdr = pp_hdr<T>(kb);
    T const* crow = gbuf + pk * E + hdr + kb;
    R best = R(-1);
    int64_t bg = -1;
    int w = -1;
    for (int e = 0; e < np; ++e) {
        T* en = const_cast<T*>(gbuf + e * E);
        R v = pp_val(en);
        int64_t gi = pp_gid(en);
        if (gi < 0) continue;
        if (v > best || (v == best && gi < bg)) { best = v; bg = gi; w = e; }
    }
    int64_t piv = w < 0 ? kk + j : bg;
    auto a1 = [](T x) { return std::abs(std::real(x)) + std::abs(std::imag(x)); };
    if (w >= 0 && thresh < 1.0 && piv != kk + j && a1(crow[j]) >= R(thresh) * best) { piv = kk + j; w = -1; }
    pip[j] = piv - kk;
    if (info && best == R(0) && *info == 0) *info = int(info_off + j + 1);
    T const* prow = w >= 0 ? gbuf + w * E + hdr : crow;
    std::vector<T> pr(prow, prow + kb), cr(crow, crow + kb);   // gbuf rows may alias nothing, copy anyway
    const bool swap = piv != kk + j;
    const int64_t lp = (swap && kd::rd_owner(d, piv) == d.myrow) ? kd::rd_lrow(d, piv) - lr_k : -1;
    if (is_pk) for (int64_t cc = 0; cc < kb; ++cc) ap[j + cc * lda] = pr[cc];
    if (lp >= 0) for (int64_t cc = 0; cc < kb; ++cc) ap[lp + cc * lda] = cr[cc];
    const T ujj = pr[j];
    for (int64_t r = r_upd0; r < mr; ++r) {
        T l = ujj != T(0) ? ap[r + j * lda] / ujj : ap[r + j * lda];
        ap[r + j * lda] = l;
        for (int64_t cc = j + 1; cc < cend; ++cc) ap[r + cc * lda] -= l * pr[cc];
    }
}

template <typename T>
void panel_xfer(lb::Ctx const& c, int64_t M, int64_t kb, int64_t kk, RowDist const& d, PanelBases const& pb,
                int64_t maxr, T* G, T* P, int64_t ldp, T* ap, int64_t lda, int mode) {
    if (M <= 0 || kb <= 0) return;
    if (c.dev()) {
        kd::panel_xfer(M, kb, kk, d, pb, maxr, dptr(G), dptr(P), ldp, dptr(ap), lda, mode, c.stream);
        return;
    }
    for (int64_t i = 0; i < M; ++i) {
        const int64_t R = d.row0 + kk + i;
        const int r = int((R / d.mb + d.rsrc) % d.p);
        const int64_t t = (R / d.mb / d.p) * d.mb + R % d.mb - pb.base[r];
        if (mode == 0) {
            for (int64_t j = 0; j < kb; ++j) P[i + j * ldp] = G[r * maxr * kb + t + j * maxr];
        } else if (r == d.myrow) {
            for (int64_t j = 0; j < kb; ++j) ap[t + j * lda] = P[i + j * ldp];
        }
    }
}

#define SLATE_LUDIST_INST(T)                                                                                    \
    template int64_t pplu_entry<T>(int64_t);                                                                   \
    template void pplu_cand<T>(lb::Ctx const&, int64_t, int64_t, int64_t, T const*, int64_t, int64_t,        \
                               RowDist const&, int64_t, bool, T*);                                             \
    template void pplu_apply<T>(lb::Ctx const&, int, T const*, int64_t, int64_t, int64_t, int64_t, int64_t, T*, \
                                int64_t, RowDist const&, int64_t, int64_t, int, double, bool, int64_t*, int*,  \
                                int64_t);                                                                      \
    template void gather_rows_ids<T>(lb::Ctx const&, int64_t, int64_t, int64_t const*, T const*, int64_t, T*,  \
                                     int64_t, int64_t const*, int64_t*, RowDist const&, int64_t);              \
    template void slots_pack<T>(lb::Ctx const&, int, int, int64_t, int64_t const*, T const*, int64_t,          \
                                RowDist const&, T*, int64_t);                                                  \
    template void slots_unpack<T>(lb::Ctx const&, int, int, int64_t, int64_t const*, T const*, int64_t, T*,    \
                                  int64_t, RowDist const&);                                                    \
    template void lu_sign<T>(lb::Ctx const&, int64_t, T*, int64_t, T*);                                         \
    template void panel_xfer<T>(lb::Ctx const&, int64_t, int64_t, int64_t, RowDist const&, PanelBases const&,    \
                                int64_t, T*, T*, int64_t, T*, int64_t, int);

SLATE_LUDIST_INST(float)
SLATE_LUDIST_INST(double)
SLATE_LUDIST_INST(std::complex<float>)
SLATE_LUDIST_INST(std::complex<double>)

}  // namespace ludist
}  // namespace internal
}  // namespace slate
