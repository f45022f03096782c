#!/usr/bin/env python3
"""Benchmark: rows/sec per IRLS iteration (+ time-to-converge) for the sparkGLM glm() hot path.

Workload (BASELINE.json configs[1]): binomial/logit GLM on a dense fp64 design of
100M rows x 256 columns per MI355X, resident in HBM, generated on the device by the
seeded synthetic generator (sparkglm_amd.synth; bit-identical host copy).  A "step" is
one IRLS iteration: the fused pass over every resident row (eta, mu, w, z, deviance and
the X'WX / X'Wz Gramian on fp64 MFMA) + the all-reduce over ranks + the p x p solve.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--rows R] [--p P]

N > 1 is launched by torch.distributed.run (one process per GPU); each rank holds its
own 100M-row shard (weak scaling) and the per-iteration Gram all-reduce runs on RCCL
over xGMI inside the engine.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X fp64 matrix, dense (datasheet; equal to the fp64 vector rate)
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "rows/sec per IRLS iteration + time-to-converge, 1/2/4/8 MI355X"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(p: int, seed: int, rows: int, threads: int) -> dict:
    """The CPU restatement (oracle/, test infrastructure) timed on a bounded sample."""
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import pyoracle  # noqa: E402  (checker / CPU baseline only)
    from sparkglm_amd import synth

    X, y, _, _ = synth.generate(0, 0, rows, p, seed)
    t0 = time.perf_counter()
    fit = pyoracle.fit_glm(X, y, "binomial", "logit", npart=threads, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": rows * fit.iter / dt, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": f"CPU restatement of fitMultipleBinomial (oracle/sglm_oracle.c, -O3 AVX2, OpenMP), "
                      f"{rows} x {p} logit rows of the same generator, {threads} partitions/threads, "
                      f"{fit.iter} IRLS iterations to convergence in {dt:.2f} s (not the JVM)",
            "time_to_converge_s": dt, "iters": fit.iter}


def pmc_traffic(p: int, n: int):
    """Per-launch HBM bytes of the fused pass: the per-row FETCH_SIZE + WRITE_SIZE measured by
    rocprofv3 --pmc (profiles/pmc_traffic.json, corrected as MI355X_MICROARCH.md prescribes)
    times the rows of this launch (the pass streams every row exactly once)."""
    path = os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            e = json.load(f).get(str(p))
        return None if e is None else e["bytes_per_row"] * n
    except (OSError, ValueError, KeyError):
        return None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=100_000_000, help="rows per GPU")
    ap.add_argument("--p", type=int, default=256)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--cpu-rows", type=int, default=2_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--comm", choices=["rccl", "torch"], default="rccl")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")

    import torch
    import torch.distributed as dist
    from sparkglm_amd import Engine

    dist_on = world > 1
    if dist_on:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()

    n, p = args.rows, args.p
    eng = Engine(local)
    t0 = time.perf_counter()
    eng.synth(0, rank * n, n, p, args.seed)  # this rank's shard of the global design
    gen_s = time.perf_counter() - t0
    if dist_on:
        if args.comm == "rccl":
            uid = [Engine.rccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            eng.set_comm_rccl(world, rank, uid[0])
        else:
            from sparkglm_amd.distributed import torch_allreduce
            eng.set_comm(torch_allreduce(), on_device=True)
    log(f"[rank {rank}] shard {n} x {p} generated in {gen_s:.2f} s")

    # time-to-converge: a full fit (data resident), reference semantics (tol 1e-6)
    barrier()
    t0 = time.perf_counter()
    fit = eng.fit_glm("binomial", "logit", tol=1e-6)
    barrier()
    ttc = time.perf_counter() - t0
    log(f"[rank {rank}] converged in {fit.iter} iterations, {ttc:.3f} s, deviance {fit.deviance!r}")

    beta = np.zeros(p)
    if args.warmup > 0:
        beta, _ = eng.irls_iterations(beta, args.warmup)
    eng.reset_stats()
    barrier()
    t0 = time.perf_counter()
    beta, dev = eng.irls_iterations(beta, args.steps)
    barrier()
    dt = time.perf_counter() - t0
    st = eng.stats()
    if dist_on:
        tt = torch.tensor([dt, ttc], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt, ttc = float(tt[0]), float(tt[1])

    if rank == 0:
        total_rows = n * world
        kern_ms = st["pass_kernel_ms"] / max(st["passes"], 1)
        flops = n * (p * (p + 1) + 2 * p)  # SYRK-convention X'WX + X'Wz per launch
        achieved = flops / (kern_ms * 1e-3) / 1e12
        traffic = pmc_traffic(p, n)
        out = {
            "metric": METRIC,
            "value": total_rows * args.steps / dt,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded counter-based generator, generated in HBM)",
            "config": {"workload": "binomial/logit glm, dense fp64 design, IRLS (BASELINE configs[1])",
                       "rows_per_gpu": n, "p": p, "global_rows": total_rows, "parallelism": f"rows{world}",
                       "family": "binomial", "link": "logit", "tol": 1e-6},
            "time_to_converge_s": ttc,
            "iters_to_converge": fit.iter,
            "deviance": fit.deviance,
            "roofline": {"bound": "mfma", "kernel": "irls_pass_kernel<16,binomial,logit>",
                         "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / FP64_MFMA_PEAK_TFLOPS, "traffic": traffic,
                         "kernel_ms": kern_ms, "algorithmic_flops_per_launch": flops,
                         "hbm_gbs_algorithmic": n * 8 * (p + 1) / (kern_ms * 1e-3) / 1e9},
            "breakdown_ms_per_step": {"fused_pass": kern_ms,
                                      "reduce": st["reduce_kernel_ms"] / max(st["passes"], 1),
                                      "solve": st["solve_ms"] / args.steps,
                                      "comm": st["comm_ms"] / args.steps},
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(p, args.seed, args.cpu_rows, threads)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
