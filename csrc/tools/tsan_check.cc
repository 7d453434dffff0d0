// ThreadSanitizer driver for the threaded runtime, host target (`make tsan`,
// tests/test_build.py): in-process ranks (run_in_process + ThreadComm: host
// rendezvous, condition variables, peer copies), the DAG scheduler's lanes
// (p x q LU / Cholesky / QR with lookahead 1 and 2, whose tasks run on the
// scheduler's host threads) and tile send / recv / bcast between ranks.
// Every rank checks its results; exit 0 only if every check passed.  Data
// races are reported by TSan itself (TSAN_OPTIONS=halt_on_error=1 makes the
// first one fatal).
#include "slate_amd/slate.hh"
#include "slate_amd/inproc.hh"

#include <atomic>
#include <cmath>
#include <cstdio>
#include <string>

using namespace slate;

namespace {

std::atomic<int> g_fail{0};

void check(bool ok, const char* what, int rank) {
    if (!ok) {
        std::fprintf(stderr, "rank %d: %s FAILED\n", rank, what);
        ++g_fail;
    }
}

Options host(int64_t la) { return {{Option::Target, Target::HostTask}, {Option::Lookahead, la}}; }

template <typename T>
void fill(Matrix<T>& A, uint64_t seed, bool spd = false) {
    A.insertLocalTiles(Target::HostTask);
    BaseMatrix<T>& B = A;
    generate_matrix(std::string(spd ? "spd" : "rand"), B, seed, -1, host(1));
}

/// ||B - A X||_1 / (n ||A||_1 ||X||_1)
double residual(Matrix<double> const& A, Matrix<double> const& X, Matrix<double> const& B) {
    Matrix<double> R = B.emptyLike();
    R.insertLocalTiles(Target::HostTask);
    copy<double, double>(B, R, host(1));
    gemm(-1.0, A, X, 1.0, R, host(1));
    return norm(Norm::One, R, host(1)) /
           (double(A.n()) * norm(Norm::One, A, host(1)) * norm(Norm::One, X, host(1)));
}

void rank_body(int rank, GridPtr const& g) {
    const int64_t n = 192, nb = 32, nrhs = 3;
    for (int64_t la : {1, 2}) {
        auto o = host(la);
        // LU (partial and tournament pivoting) + solve
        for (int64_t method : {int64_t(MethodLU::PartialPiv), int64_t(MethodLU::CALU)}) {
            Matrix<double> A(n, n, nb, g), B(n, nrhs, nb, g);
            fill(A, 11);
            fill(B, 12);
            Matrix<double> A0 = A.emptyLike(), B0 = B.emptyLike();
            A0.insertLocalTiles(Target::HostTask);
            B0.insertLocalTiles(Target::HostTask);
            copy<double, double>(A, A0, o);
            copy<double, double>(B, B0, o);
            Pivots piv;
            Options om = o;
            om[Option::MethodLU] = method;
            int64_t info = gesv(A, piv, B, om);
            check(info == 0 && residual(A0, B, B0) < 1e-13, "gesv", rank);
        }
        // Cholesky
        {
            Matrix<double> A(n, n, nb, g), B(n, nrhs, nb, g);
            fill(A, 21, true);
            fill(B, 22);
            Matrix<double> A0 = A.emptyLike(), B0 = B.emptyLike();
            A0.insertLocalTiles(Target::HostTask);
            B0.insertLocalTiles(Target::HostTask);
            copy<double, double>(A, A0, o);
            copy<double, double>(B, B0, o);
            HermitianMatrix<double> H(Uplo::Lower, A);
            int64_t info = posv(H, B, o);
            check(info == 0 && residual(A0, B, B0) < 1e-13, "posv", rank);
        }
        // QR + least squares residual orthogonality: ||A^H (b - A x)|| small
        {
            Matrix<double> A(2 * n, n, nb, g), B(2 * n, 1, nb, g);
            fill(A, 31);
            fill(B, 32);
            Matrix<double> A0 = A.emptyLike();
            A0.insertLocalTiles(Target::HostTask);
            copy<double, double>(A, A0, o);
            TriangularFactors<double> T;
            geqrf(A, T, o);
            Matrix<double> C = A0.emptyLike();
            C.insertLocalTiles(Target::HostTask);
            copy<double, double>(A0, C, o);
            unmqr(Side::Left, Op::ConjTrans, A, T, C, o);
            // Q^H A0 below the first n rows must vanish
            double below = norm(Norm::Max, Matrix<double>(C.slice(n, 2 * n - 1, 0, n - 1)), o);
            check(below < 1e-12 * n, "geqrf / unmqr", rank);
        }
    }
    // tile-level point-to-point and broadcast between ranks
    {
        Matrix<double> A(4 * nb, 4 * nb, nb, g);
        fill(A, 41);
        const int src = A.tileRank(0, 0);
        const int dst = A.tileRank(1, 1);
        if (src != dst) {
            if (g->rank() == src) A.tileSend(0, 0, dst);
            if (g->rank() == dst) A.tileRecv(0, 0, src);
        }
        A.tileBcast(2, 0, A.sub(2, 2, 0, 3));
    }
}

}  // namespace

int main() {
    for (auto pq : {std::pair<int, int>{1, 2}, {2, 2}, {2, 1}}) {
        run_in_process(pq.first, pq.second, rank_body);
        std::printf("grid %d x %d: %s\n", pq.first, pq.second, g_fail ? "FAILED" : "ok");
    }
    std::printf("%s\n", g_fail ? "TSAN_CHECK FAILED" : "TSAN_CHECK OK");
    return g_fail ? 1 : 0;
}
