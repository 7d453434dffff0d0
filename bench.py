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

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import slate_d35_amd as s  # noqa: E402
from slate_d35_amd.utils import flops as F  # noqa: E402

METRIC = "fp64 TFLOP/s (whole node) for dgemm / dpotrf / dgetrf / dgeqrf, n=64k, at 1/2/4/8 MI355X"
ALL = ["dgemm", "dpotrf", "dgetrf", "dgeqrf"]
EXTRA = ["dgesv_mixed"]  # BASELINE config 5; run with --routines dgesv_mixed


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
    ap.add_argument("--lookahead", type=int, default=1)
    ap.add_argument("--method-lu", default="tntpiv", choices=["ppiv", "tntpiv"])
    ap.add_argument("--trace", default="")
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if s.device_available():
        s._slate.set_device(int(os.environ.get("LOCAL_RANK", "0")) % max(1, s._slate.device_count()))
    target = "d" if s.device_available() else "h"
    p, q = (a.p, a.q) if a.p and a.q else s.choose_grid(world)
    grid = s.init_grid(p, q)
    n = a.n
    # Default tiles: 512 everywhere, except on one GPU where dgetrf / dpotrf
    # run 2-4% faster at nb = 1024 (profiles/nb_sweep_r1_n65536_1gpu.txt:
    # getrf 50.3 -> 52.3, potrf 57.8 -> 58.6 TFLOP/s); dgeqrf stays at 512
    # (384: 50.5, 512: 51.9).  Multi-GPU grids keep 512 so the 2-D cyclic
    # distribution has enough block columns per process.
    # dgesv_mixed likewise (fp32 LU: 2.49 -> 2.42 s, profiles/r1_gesv_mixed_n64k_norm_fix.txt).
    default_nb = {"dgetrf": 1024, "dpotrf": 1024, "dgesv_mixed": 1024} if world == 1 else {}
    if a.nb:
        default_nb = {}
    a.nb = a.nb or 512
    nb_per = dict(default_nb)
    nb_per.update({k: int(v) for k, v in (kv.split("=") for kv in a.nb_per.split(",") if kv)})
    opts = dict(target=target, lookahead=a.lookahead)

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

    results = {}
    routines = [r.strip() for r in a.routines.split(",") if r.strip()]
    for rname in routines:
        mats = {}
        nb = nb_per.get(rname, a.nb)
        if rname == "dgemm":
            for key, seed in (("A", 1), ("B", 2), ("C", 3)):
                M = s.Matrix(n, n, nb, np.float64, grid)
                M.insertLocalTiles(s.target_of(target))
                s._slate.generate_matrix_d("rands", M, seed, -1.0, s.opts(target))
                mats[key] = M
            flops = F.gemm_flops(n, n, n)
        elif rname == "dgesv_mixed":
            # fp32 LU + fp64 refinement; flops counted as the fp64 LU (tester convention)
            for key, seed in (("B", 7), ("X", 0)):
                M = s.Matrix(n, 1, nb, np.float64, grid)
                M.insertLocalTiles(s.target_of(target))
                s._slate.generate_matrix_d("rands", M, seed + 1, -1.0, s.opts(target))
                mats[key] = M
            M = s.Matrix(n, n, nb, np.float64, grid)
            M.insertLocalTiles(s.target_of(target))
            mats["A"] = M
            flops = F.getrf_flops(n)
        else:
            M = s.Matrix(n, n, nb, np.float64, grid)
            M.insertLocalTiles(s.target_of(target))
            mats["A"] = M
            flops = {"dpotrf": F.potrf_flops, "dgetrf": F.getrf_flops, "dgeqrf": F.geqrf_flops}[rname](n)
        times = []
        for step in range(a.warmup + a.steps):
            if rname != "dgemm":
                # diagonally dominant for dgesv_mixed so fp32 LU + refinement converges
                kind = "spd" if rname == "dpotrf" else ("diag_dominant" if rname == "dgesv_mixed" else "rands")
                s._slate.generate_matrix_d(kind, mats["A"], 100 + step, -1.0, s.opts(target))
            barrier_sync()
            if a.trace and step == a.warmup:
                s.trace.on()
            t0 = time.perf_counter()
            if rname == "dgemm":
                s.gemm(1.0, mats["A"], mats["B"], 0.0, mats["C"], **opts)
            elif rname == "dpotrf":
                info = s.potrf(s.HermitianMatrix(s.Uplo.Lower, mats["A"]), **opts)
                assert info == 0, f"dpotrf info={info}"
            elif rname == "dgetrf":
                if a.method_lu == "tntpiv":
                    info, _ = s.getrf_tntpiv(mats["A"], **opts)
                else:
                    info, _ = s.getrf(mats["A"], **opts)
                assert info == 0, f"dgetrf info={info}"
            elif rname == "dgeqrf":
                s.geqrf(mats["A"], **opts)
            elif rname == "dgesv_mixed":
                s._slate.clear_timers()
                lu = {"tntpiv": 2, "ppiv": 1}[a.method_lu]  # MethodLU::CALU / PartialPiv
                info, _, iters = s.gesv_mixed(mats["A"], mats["B"], mats["X"], method_lu=lu, **opts)
                assert info == 0 and iters >= 0, f"dgesv_mixed info={info} iters={iters}"
                if rank == 0:
                    tm = {k: round(v * 1e3, 1) for k, v in s._slate.timers().items() if "gesv_mixed" in k}
                    print(f"# dgesv_mixed iters={iters} phase ms: {tm}", file=sys.stderr, flush=True)
            barrier_sync()
            dt = time.perf_counter() - t0
            if a.trace and step == a.warmup:
                s.trace.finish(grid.world, f"{a.trace}_{rname}")
                s.trace.off()
            if step >= a.warmup:
                times.append(dt)
            if rank == 0:
                print(f"# {rname} step {step} {'warm' if step < a.warmup else 'timed'}: {dt*1e3:.1f} ms "
                      f"{flops/dt/1e12:.2f} TFLOP/s", file=sys.stderr, flush=True)
        t = max_over_ranks(float(np.mean(times)))
        results[rname] = {"ms": t * 1e3, "tflops": flops / t / 1e12, "flops": flops, "nb": nb}
        del mats
        s.sync()
        s._slate.release_cache()

    tot_flops = sum(r["flops"] for r in results.values())
    tot_t = sum(r["ms"] for r in results.values()) / 1e3
    value = tot_flops / tot_t / 1e12
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
        "data": "synthetic (counter-hash uniform[-1,1); SPD = symmetric + n*I for dpotrf)",
        "config": {
            "model": "+".join(f"{k}(nb={v['nb']})" for k, v in results.items()) + f" n={n}",
            "global_batch": 1,
            "seq_len": n,
            "parallelism": f"2d-block-cyclic {p}x{q} (one process per GPU, RCCL)" if world > 1 else "1x1",
            "lookahead": a.lookahead,
            "lu_method": a.method_lu,
        },
        "routines": {k: {"tflops": round(v["tflops"], 3), "ms": round(v["ms"], 2)} for k, v in results.items()},
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        del grid
        s.finalize()


if __name__ == "__main__":
    main()
