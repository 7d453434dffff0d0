#!/usr/bin/env python3
"""Headline benchmark: fp64 TFLOP/s (whole node) for dgemm / dpotrf / dgetrf /
dgeqrf at n = 65536 on N MI355X GPUs (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU; a p x q process grid (1x1, 1x2, 2x2, 2x4 by default)
with RCCL communicators.  Each step runs every routine once on a freshly
generated synthetic random matrix (counter-hash generator on the device,
outside the timed region); each routine call is bracketed by a barrier and a
device synchronize, the per-routine time is the MAX over ranks of the mean
over the K timed steps.  `value` = total flops / total time over the routine
suite (whole-job aggregate); per-routine TFLOP/s are in `routines`.
Flops are LAWN-41 counts (reference docs/latex/flops.py), as the reference
tester reports them.
"""
from __future__ import annotations

import time as _time

_T_START = _time.time()   # wall clock of the whole run (the driver's limit counts from launch)

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# The package (and with it the HIP runtime) is imported by the ranks only:
# a self-launching parent (launch_ranks) must not touch the GPU.
s = None
F = None


def _import_slate():
    global s, F
    import slate_d35_amd as s_  # noqa: E402
    from slate_d35_amd.utils import flops as F_  # noqa: E402
    s, F = s_, F_

METRIC = "fp64 TFLOP/s (whole node) for dgemm / dpotrf / dgetrf / dgeqrf, n=64k, at 1/2/4/8 MI355X"
ALL = ["dgemm", "dpotrf", "dgetrf", "dgeqrf"]
# Per-routine grid shapes and tile sizes by world size (absent: the job's
# p x q / --nb), chosen with the critical-path model (32 reserved CUs,
# copy-engine broadcasts; profiles/r6_critpath_8gpu_sweep.txt,
# profiles/r6_critpath_2_4gpu_sweep.txt), predicted whole-job TFLOP/s:
#   8: LU 2 x 4 nb 512 (193-194 with the 512-thread tournament tree; nb 256:
#      185-187, profiles/r6_tslu_nt.txt), QR 8 x 1 nb 512 (337; 4 x 2: 308),
#      Cholesky 8 x 1 nb 512 (321 once the lookahead column's transposed
#      tiles travel first, profiles/r6_potrf_split.txt; 4 x 2: 296)
#   4: LU 2 x 2 nb 512 (143), QR 4 x 1 nb 1024 (187; 2 x 2: 170), Cholesky
#      4 x 1 nb 1024 (187; 2 x 2: 161)
#   2: everything 2 x 1 (1 x 2 is 5-10 % lower): LU nb 1024 (92; the p > 1
#      LU takes tiles <= 1024), QR nb 1024 (97), Cholesky nb 1536 (97)
# The BASELINE configs 3-5 keep the reference's 2 x 4.
GRID_PER = {
    2: {"dgetrf": (2, 1), "dpotrf": (2, 1), "dgeqrf": (2, 1)},
    4: {"dgeqrf": (4, 1), "dpotrf": (4, 1)},
    8: {"dgeqrf": (8, 1), "dpotrf": (8, 1), "cfg4_dgeqrf_nb256": (2, 4)},
}
NB_PER_WORLD = {
    1: {"dgetrf": 2048, "dpotrf": 1536, "dgeqrf": 1024, "dgesv_mixed": 1024},
    2: {"dgetrf": 1024, "dpotrf": 1536, "dgeqrf": 1024},
    4: {"dgetrf": 512, "dpotrf": 1024, "dgeqrf": 1024},
    8: {},
}
# BASELINE.json configs beyond the 4-routine headline suite (run after it,
# reported under "configs"): name -> (routine, n or None = --dim, nb, target)
EXTRAS = {
    "cfg1_dgemm_host_n2048_nb256": ("dgemm", 2048, 256, "h"),
    "cfg2_dpotrf_n32768_nb512": ("dpotrf", -2, 512, None),       # -2: half of --dim (32768 at the default)
    # config 3: the reference's 8-GPU tournament LU, 2 x 4, nb 512 (multi-GPU jobs only)
    "cfg3_dgetrf_tntpiv_nb512": ("dgetrf", None, 512, None),
    "cfg4_dgeqrf_nb256": ("dgeqrf", None, 256, None),
    "cfg5_dgesv_mixed": ("dgesv_mixed", None, None, None),
    # the reference's semantics (src/gesv_mixed.cc:219-279): classical
    # refinement, then the fp64 fallback -- no GMRES-IR escalation
    "cfg5_dgesv_mixed_refsem": ("dgesv_mixed", None, None, None),
    # the default LU (MethodLU::PartialPiv: what gesv / LAPACK / ScaLAPACK
    # callers get), tracked next to the tournament LU of the suite
    "dgetrf_ppiv": ("dgetrf", None, 1024, None),
}


class Watchdog:
    """Fail fast on a hung step (a peer that never joins a collective): after
    the armed deadline, abort every RCCL communicator of this process (the
    stuck kernels return) and exit 124, so torchrun tears the job down and
    the run reports an error instead of holding the node until the driver's
    limit.  SLATE_BENCH_STEP_TIMEOUT (s) bounds a routine's first step and
    every generation / check phase; later steps get max(60 s, 4x the first)."""

    def __init__(self, rank):
        import threading
        self.rank, self.deadline, self.what = rank, None, ""
        self.base = float(os.environ.get("SLATE_BENCH_STEP_TIMEOUT", "300"))
        self.lock = threading.Lock()
        threading.Thread(target=self._loop, daemon=True).start()

    def arm(self, what, secs=None):
        with self.lock:
            self.what, self.deadline = what, time.time() + (secs or self.base)

    def disarm(self):
        with self.lock:
            self.deadline = None

    def _loop(self):
        import threading
        while True:
            time.sleep(1.0)
            with self.lock:
                late = self.deadline is not None and time.time() > self.deadline
                what = self.what
            if not late:
                continue
            errs = ""
            try:
                errs = s._slate.comm_async_errors()
            except Exception:
                pass
            print(f"# WATCHDOG rank {self.rank}: '{what}' exceeded its time limit; RCCL async errors: "
                  f"{errs or 'none'}; aborting communicators", file=sys.stderr, flush=True)
            t = threading.Thread(target=lambda: s._slate.comm_abort_all(), daemon=True)
            t.start()
            t.join(30)
            os._exit(124)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--dim", "--n", dest="n", type=int, default=65536)
    ap.add_argument("--nb", type=int, default=0, help="tile size for every routine (default: per-routine table)")
    ap.add_argument("--nb-per", default="", help="per-routine nb overrides, e.g. dgeqrf=256,dgetrf=512")
    ap.add_argument("--routines", default=",".join(ALL))
    ap.add_argument("--p", type=int, default=0)
    ap.add_argument("--q", type=int, default=0)
    ap.add_argument("--lookahead", type=int, default=0, help="0: per-routine default (see la_per)")
    ap.add_argument("--grid-per", default="", help="per-routine grid shapes, e.g. dgetrf=4x2,dgeqrf=2x4")
    ap.add_argument("--method-lu", default="tntpiv", choices=["ppiv", "tntpiv"])
    ap.add_argument("--trace", default="")
    ap.add_argument("--mixed-escalate", default="yes", choices=["yes", "no"],
                    help="dgesv_mixed: GMRES-IR escalation before the fp64 fallback (no = reference semantics)")
    ap.add_argument("--extras", default="all", help="BASELINE configs to add after the suite: all, none, or names")
    ap.add_argument("--check", default="yes", choices=["yes", "no"],
                    help="backward-error check of each routine after its timed steps (outside the timed region)")
    ap.add_argument("--extras-steps", type=int, default=2, help="timed steps per BASELINE extra config")
    ap.add_argument("--extras-warmup", type=int, default=1, help="warmup steps per BASELINE extra config")
    ap.add_argument("--time-budget", type=float, default=555.0,
                    help="seconds since launch after which no further extra config is started (the driver "
                         "allows 600 s per run; the headline suite itself always runs its K + W steps)")
    return ap.parse_args()


def launch_ranks(a) -> int:
    """`python bench.py --gpus N` without a launcher: start N rank processes
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT, the
    environment torchrun would give them; the reference's runner wraps itself
    in `mpirun -np N` the same way, test/run_tests.py:127-173).  This parent
    never imports the extension nor initialises the GPU, and never execs:
    the ranks are fresh child processes.  They write straight to this
    process's stdout / stderr (rank 0 prints the JSON line).  When a rank
    fails the others get a grace period (their own watchdogs fire first),
    then the whole set is killed; the exit code is the first failing rank's.
    SLATE_BENCH_FAKE_HOSTS=1 gives every rank its own NCCL_HOSTID, so that N
    ranks can rehearse the RCCL path on ONE GPU (RCCL's socket transport
    over loopback instead of refusing a duplicate device)."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    n = a.gpus
    fake = os.environ.get("SLATE_BENCH_FAKE_HOSTS", "0") == "1"
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   SLATE_MASTER_PORT=str(port), SLATE_BENCH_LAUNCHER="self")
        if fake:
            env.update(NCCL_HOSTID=f"slate-bench-host-{r}", NCCL_SOCKET_IFNAME="lo")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      start_new_session=True))

    def kill_all(sig):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    pass

    def on_term(signum, _frame):
        kill_all(signal.SIGTERM)
        raise SystemExit(128 + signum)

    signal.signal(signal.SIGTERM, on_term)
    signal.signal(signal.SIGINT, on_term)
    limit = float(os.environ.get("SLATE_BENCH_LAUNCH_TIMEOUT", "0")) or None
    grace = float(os.environ.get("SLATE_BENCH_RANK_GRACE", "60"))
    rc, failed_at = 0, None
    t0 = time.time()
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad and rc == 0:
            rc, failed_at = bad[0], time.time()
            print(f"# launcher: a rank exited with {rc}; stopping the others within {grace:.0f} s",
                  file=sys.stderr, flush=True)
        if all(c is not None for c in codes):
            break
        if failed_at is not None and time.time() - failed_at > grace:
            kill_all(signal.SIGKILL)
        if limit and time.time() - t0 > limit:
            print(f"# launcher: time limit {limit:.0f} s reached; killing the ranks", file=sys.stderr, flush=True)
            kill_all(signal.SIGKILL)
            rc = rc or 124
        time.sleep(0.2)
    for p in procs:
        p.wait()
    return rc


def comm_info(grid, world):
    """What the communicators actually created report: transport name and
    sizes (RCCL: ncclCommCount), plus every rank's HIP device
    (ncclCommCuDevice for RCCL comms, else the process's current device)."""
    info = {"backend": "self" if world == 1 else grid.world.name(), "world": grid.world.size() if world > 1 else 1,
            "row": grid.row_comm.size() if world > 1 else 1, "col": grid.col_comm.size() if world > 1 else 1,
            "grid": [grid.p, grid.q]}
    dev = s._slate.get_device() if s.device_available() else -1
    if world > 1:
        d = grid.world.device()
        dev = d if d >= 0 else dev
        v = [0] * world
        v[grid.world.rank()] = dev + 1
        info["devices"] = [x - 1 for x in grid.world.allreduce_sum_i64(v)]
        info["fast_lane"] = bool(grid.has_fast_lane)
    else:
        info["devices"] = [dev]
    info["launcher"] = os.environ.get("SLATE_BENCH_LAUNCHER", "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ
                                      else ("env" if world > 1 else "none"))
    return info


def main(a):
    _import_slate()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if s.device_available():
        s._slate.set_device(int(os.environ.get("LOCAL_RANK", "0")) % max(1, s._slate.device_count()))
    target = "d" if s.device_available() else "h"
    p, q = (a.p, a.q) if a.p and a.q else s.choose_grid(world)
    wd = Watchdog(rank)
    wd.arm("init_grid")
    grid = s.init_grid(p, q)
    comm = comm_info(grid, world)
    wd.disarm()
    if rank == 0:
        print(f"# comm: {json.dumps(comm)}", file=sys.stderr, flush=True)
    n = a.n
    # Default tiles: 512 everywhere, except on one GPU where dgetrf / dpotrf
    # run 2-4% faster at nb = 1024 (profiles/nb_sweep_r1_n65536_1gpu.txt:
    # getrf 50.3 -> 52.3, potrf 57.8 -> 58.6 TFLOP/s); dgeqrf stays at 512
    # (384: 50.5, 512: 51.9).  Multi-GPU grids keep 512 so the 2-D cyclic
    # distribution has enough block columns per process.
    # dgesv_mixed likewise (fp32 LU: 2.49 -> 2.42 s, profiles/r1_gesv_mixed_n64k_norm_fix.txt).
    # Round 3: dgetrf at nb = 2048 once tiles wider than 1024 factor correctly
    # (LDS-staged row permutation): 3370 -> 3283-3299 ms at n = 65536
    # (profiles/r3_nb_sweep.txt); dgeqrf 512 vs 1024 and dpotrf 1024 vs 2048
    # measured equal on one box.
    # Round 5 (single-wave leaf kernels make wide diagonal blocks cheap):
    # dpotrf 1536 vs 1024 62.7-63.0 -> 63.3-63.4, dgeqrf 1024 vs 512 59.2 ->
    # 59.8-59.9 TFLOP/s, interleaved on one box (profiles/r5_nb_ab.txt).
    # p x q: NB_PER_WORLD (the critical-path sweeps)
    default_nb = dict(NB_PER_WORLD.get(world, {}))
    if a.nb:
        default_nb = {}
    a.nb = a.nb or 512
    nb_per = dict(default_nb)
    nb_per.update({k: int(v) for k, v in (kv.split("=") for kv in a.nb_per.split(",") if kv)})
    # Lookahead: 1 (the reference default), except on one GPU where dpotrf and
    # dgeqrf measured faster at 2 (profiles/r2_sweep2_la_nb_ppiv.txt: potrf
    # 59.4 -> 60.1, geqrf 55.7 -> 56.2 TFLOP/s at n=65536).
    # p x q grids: lookahead 2 for every factorization, so one late panel
    # (its chain of tournament / CholeskyQR kernels and messages is longer
    # than a step's trailing update for most steps at 2 x 4,
    # profiles/r4_critpath_2x4_*.txt) does not stall the trailing queue of
    # the next step as well.
    # Round 5: dgetrf at 2 on one GPU too (58.65-58.85 -> 58.89-59.00 TFLOP/s,
    # interleaved, profiles/r5_lookahead_ab.txt).
    la_per = ({"dpotrf": 2, "dgeqrf": 2, "dgetrf": 2} if world == 1
              else {"dpotrf": 2, "dgeqrf": 2, "dgetrf": 2, "dgesv_mixed": 2})

    def la_of(rname):
        return a.lookahead or la_per.get(rname, 1)

    # Grid shape per routine on p x q > 1 (--grid-per dgetrf=4x2,...; the
    # defaults come from the 8-GPU critical-path sweep,
    # profiles/r6_critpath_8gpu_sweep.txt): extra grids are split from the
    # same world communicator, created on first use in the same order on
    # every rank.
    grid_per = dict(GRID_PER.get(world, {}))
    grid_per.update({k: tuple(int(x) for x in v.split("x")) for k, v in
                     (kv.split("=") for kv in a.grid_per.split(",") if kv)})
    grids = {(grid.p, grid.q): grid}

    def grid_for(label, rname):
        shape = grid_per.get(label) or grid_per.get(rname)
        if world == 1 or shape is None or a.p:
            return grid
        if shape not in grids:
            grids[shape] = s.parallel.reshape_grid(*shape)
        return grids[shape]

    def barrier_sync():
        s.sync()
        if world > 1:
            grid.world.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        import torch
        import torch.distributed as dist
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def residual(rname, mats, kind, seed, nb, n_, tg, grid):
        """Backward error of the result just computed (reference tester
        formulas, test/test_gesv.cc:330-377, test_posv.cc:302-343):
        ||b - A x|| / (||A|| ||x|| n eps) for the solves, and
        ||C x - A (B x)|| / (||A|| ||B|| ||x|| n eps) for gemm."""
        eps = np.finfo(np.float64).eps
        tgt = s.target_of(tg)

        def vec(seed_):
            V = s.Matrix(n_, 1, nb, np.float64, grid)
            V.insertLocalTiles(tgt)
            s._slate.generate_matrix_d("rands", V, seed_, -1.0, s.opts(tg))
            return V

        def inf(M):
            return s.norm(s.Norm.Inf, M, target=tg)

        o = dict(target=tg)
        if rname == "dgemm":
            x = vec(901)
            y1, t, y2 = vec(0), vec(0), vec(0)
            s.gemm(1.0, mats["C"], x, 0.0, y1, **o)
            s.gemm(1.0, mats["B"], x, 0.0, t, **o)
            s.gemm(1.0, mats["A"], t, 0.0, y2, **o)
            s.add(-1.0, y2, 1.0, y1, **o)
            return inf(y1) / (inf(mats["A"]) * inf(mats["B"]) * inf(x) * n_ * eps)
        # original matrix (the generator is deterministic), right-hand side b
        A0 = s.Matrix(n_, n_, nb, np.float64, grid)
        A0.insertLocalTiles(tgt)
        s._slate.generate_matrix_d(kind, A0, seed, -1.0, s.opts(tg))
        b = vec(902)
        if rname == "dgesv_mixed":
            X = mats["X"]
            b = mats["B"]
        else:
            X = vec(902)
            if rname == "dpotrf":
                s.potrs(s.HermitianMatrix(s.Uplo.Lower, mats["A"]), X, **o)
            elif rname == "dgetrf":
                s.getrs(mats["A"], mats["piv"], X, **o)
            elif rname == "dgeqrf":
                s.unmqr(s.Side.Left, s.Op.ConjTrans, mats["A"], mats["T"], X, **o)
                R = s.TriangularMatrix(s.Uplo.Upper, s.Diag.NonUnit, mats["A"])
                s.trsm(s.Side.Left, 1.0, R, X, **o)
        # r = b - A0 X
        r = vec(0)
        s.gemm(-1.0, A0, X, 0.0, r, **o)
        s.add(1.0, b, 1.0, r, **o)
        err = inf(r) / (inf(A0) * inf(X) * n_ * eps)
        del A0
        return err

    def run(rname, n_, nb, tg, label, warmup=None, steps=None, deadline=None):
        """W untimed + K timed steps of one routine; returns its result dict.
        With a deadline (extras only) the timed steps are cut to what fits
        after the first step's duration is known (at least one)."""
        warmup = a.warmup if warmup is None else warmup
        steps = a.steps if steps is None else steps
        mats = {}
        tgt = s.target_of(tg)
        o = dict(target=tg, lookahead=la_of(rname))
        grid_r = grid_for(label, rname)
        if rname == "dgemm":
            for key, seed in (("A", 1), ("B", 2), ("C", 3)):
                M = s.Matrix(n_, n_, nb, np.float64, grid_r)
                M.insertLocalTiles(tgt)
                s._slate.generate_matrix_d("rands", M, seed, -1.0, s.opts(tg))
                mats[key] = M
            flops = F.gemm_flops(n_, n_, n_)
        elif rname == "dgesv_mixed":
            for key, seed in (("B", 7), ("X", 0)):
                M = s.Matrix(n_, 1, nb, np.float64, grid_r)
                M.insertLocalTiles(tgt)
                s._slate.generate_matrix_d("rands", M, seed + 1, -1.0, s.opts(tg))
                mats[key] = M
            M = s.Matrix(n_, n_, nb, np.float64, grid_r)
            M.insertLocalTiles(tgt)
            mats["A"] = M
            flops = F.getrf_flops(n_)   # tester convention: counted as the fp64 LU
        else:
            M = s.Matrix(n_, n_, nb, np.float64, grid_r)
            M.insertLocalTiles(tgt)
            mats["A"] = M
            flops = {"dpotrf": F.potrf_flops, "dgetrf": F.getrf_flops, "dgeqrf": F.geqrf_flops}[rname](n_)
        # random (rands) matrices everywhere, as the reference tester; SPD for potrf
        kind = "spd" if rname == "dpotrf" else "rands"
        times, extra = [], {}
        seed = 0
        step, total = 0, warmup + steps
        first_dt = None
        while step < total:
            seed = 100 + step
            wd.arm(f"{label} generate {step}")
            if rname != "dgemm":
                s._slate.generate_matrix_d(kind, mats["A"], seed, -1.0, s.opts(tg))
            barrier_sync()
            wd.arm(f"{label} step {step}", None if first_dt is None else max(60.0, 4 * first_dt))
            if a.trace and step == warmup:
                s.trace.on()
            t0 = time.perf_counter()
            if rname == "dgemm":
                s.gemm(1.0, mats["A"], mats["B"], 0.0, mats["C"], **o)
            elif rname == "dpotrf":
                info = s.potrf(s.HermitianMatrix(s.Uplo.Lower, mats["A"]), **o)
                assert info == 0, f"dpotrf info={info}"
            elif rname == "dgetrf":
                if a.method_lu == "tntpiv" and not label.endswith("_ppiv"):
                    info, piv = s.getrf_tntpiv(mats["A"], **o)
                else:
                    info, piv = s.getrf(mats["A"], **o)
                extra["method"] = "tntpiv" if (a.method_lu == "tntpiv" and not label.endswith("_ppiv")) else "ppiv"
                mats["piv"] = piv
                assert info == 0, f"dgetrf info={info}"
            elif rname == "dgeqrf":
                mats["T"] = s.geqrf(mats["A"], **o)
            elif rname == "dgesv_mixed":
                s._slate.clear_timers()
                lu = {"tntpiv": 2, "ppiv": 1}[a.method_lu]  # MethodLU::CALU / PartialPiv
                # GMRES-IR escalation on the same fp32 factors when classical
                # refinement stalls (Option::EscalateGmres; the fp64 fallback
                # stays behind it): a random n = 65536 matrix is sometimes too
                # ill-conditioned for classical fp32 refinement within 30 steps
                esc = a.mixed_escalate == "yes" and not label.endswith("_refsem")
                info, piv, iters = s.gesv_mixed(mats["A"], mats["B"], mats["X"], method_lu=lu,
                                                escalate_gmres=esc, **o)
                mats["piv"] = piv
                assert info == 0, f"dgesv_mixed info={info} iters={iters}"
                if step >= warmup:
                    extra.setdefault("iterations_per_step", []).append(int(iters))
                    extra["iterations"] = int(iters)
                    extra["fallback"] = bool(extra.get("fallback", False) or iters < 0)
                    extra["escalate_gmres"] = esc
                    extra.setdefault("fallback_per_step", []).append(bool(iters < 0))
                if rank == 0:
                    tm = {k: round(v * 1e3, 1) for k, v in s._slate.timers().items()
                          if "gesv_mixed" in k or "gmres" in k}
                    print(f"# dgesv_mixed iters={iters} phase ms: {tm}", file=sys.stderr, flush=True)
            barrier_sync()
            dt = time.perf_counter() - t0
            wd.disarm()
            if first_dt is None:
                first_dt = dt
            if a.trace and step == warmup:
                s.trace.finish(grid_r.world, f"{a.trace}_{label}")
                s.trace.off()
                s.trace.clear()
            if step >= warmup:
                times.append(dt)
            if rank == 0:
                print(f"# {label} step {step} {'warm' if step < warmup else 'timed'}: {dt*1e3:.1f} ms "
                      f"{flops/dt/1e12:.2f} TFLOP/s", file=sys.stderr, flush=True)
            step += 1
            if deadline is not None and step == 1:
                # steps that still fit (same decision on every rank)
                left = -max_over_ranks(-(deadline - (time.time() - _T_START)))
                fit = int(left // (max_over_ranks(dt) * 1.15))
                total = min(total, max(warmup + 1, step + fit))
        t = max_over_ranks(float(np.mean(times)))
        res = {"ms": t * 1e3, "tflops": flops / t / 1e12, "flops": flops, "nb": nb, "n": n_,
               "grid": f"{grid_r.p}x{grid_r.q}", "lookahead": la_of(rname),
               "steps": len(times), "warmup": warmup}
        if a.check == "yes":
            wd.arm(f"{label} residual check")
            err = residual(rname, mats, kind, seed, nb, n_, tg, grid_r)
            wd.disarm()
            res["backward_error"] = float(f"{err:.3e}")
            res["check"] = "pass" if err < 50 else "FAIL"
            if rank == 0:
                print(f"# {label} backward error {err:.3e} ({res['check']})", file=sys.stderr, flush=True)
        res.update(extra)
        del mats
        s.sync()
        s._slate.release_cache()
        return res

    results = {}
    routines = [r.strip() for r in a.routines.split(",") if r.strip() and r.strip() != "none"]
    for rname in routines:
        results[rname] = run(rname, n, nb_per.get(rname, a.nb), target, rname)
    configs = {}
    extras = list(EXTRAS) if a.extras == "all" else ([] if a.extras == "none" else a.extras.split(","))
    # per-flop time of the slowest suite routine: first-step estimate for an extra
    rate = max((r["ms"] / 1e3 / r["flops"] for r in results.values()), default=0.0)
    for name in extras:
        rname, n_, nb_, tg_ = EXTRAS[name]
        tg_ = tg_ or target
        if tg_ == "h" and world > 1:
            continue   # config 1 is a one-process host-target plumbing check
        if name.startswith("cfg3") and world == 1:
            continue   # config 3 is the 2 x 4 LU (the 1-GPU suite's dgetrf covers one GPU)
        nb_ = nb_per.get(name) or nb_ or nb_per.get(rname, a.nb)   # --nb-per <extra name>=nb overrides
        n_ = n if n_ is None else (n // 2 if n_ == -2 else n_)
        fl = {"dgemm": F.gemm_flops(n_, n_, n_), "dpotrf": F.potrf_flops(n_), "dgeqrf": F.geqrf_flops(n_)}.get(
            rname, F.getrf_flops(n_))
        # the first step, its residual check and the matrix generation must fit
        need = 2.5 * fl * rate + 5.0 if tg_ != "h" else 5.0
        elapsed = max_over_ranks(time.time() - _T_START)
        if elapsed + need > a.time_budget:
            configs[name] = {"skipped": f"time budget: {elapsed:.0f} s elapsed, ~{need:.0f} s needed, "
                                        f"budget {a.time_budget:.0f} s"}
            if rank == 0:
                print(f"# {name} skipped ({configs[name]['skipped']})", file=sys.stderr, flush=True)
            continue
        configs[name] = run(rname, n_, nb_, tg_, name, warmup=a.extras_warmup, steps=a.extras_steps,
                            deadline=a.time_budget)

    tot_flops = sum(r["flops"] for r in results.values())
    tot_t = sum(r["ms"] for r in results.values()) / 1e3
    value = tot_flops / tot_t / 1e12 if tot_t > 0 else 0.0   # (--routines none: extras only)
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "TFLOP/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(tot_t * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp64",
        "data": "synthetic random (rands: counter-hash uniform[-1,1); SPD = symmetric + n*I for dpotrf)",
        "config": {
            "model": "+".join(f"{k}(nb={v['nb']}" + (f", {v['grid']}" if v["grid"] != f"{p}x{q}" else "") + ")"
                              for k, v in results.items()) + f" n={n}",
            "global_batch": 1,
            "seq_len": n,
            "parallelism": (f"2d-block-cyclic {p}x{q} (one process per GPU, {comm['backend']})" if world > 1
                            else "1x1"),
            "comm": comm,
            "lookahead": {k: la_of(k) for k in results} if not a.lookahead else a.lookahead,
            "lu_method": a.method_lu,
        },
        "routines": {k: {kk: (round(vv, 4) if isinstance(vv, float) and kk != "backward_error" else vv)
                         for kk, vv in v.items() if kk != "flops"} for k, v in results.items()},
        "configs": {k: {kk: (round(vv, 4) if isinstance(vv, float) and kk != "backward_error" else vv)
                        for kk, vv in v.items() if kk != "flops"} for k, v in configs.items()},
        "wall_s": round(time.time() - _T_START, 1),
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        del grid
        s.finalize()


if __name__ == "__main__":
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    main(args)
