#!/usr/bin/env python3
"""Benchmark: rows/sec per IRLS iteration (+ time-to-converge) for the sparkGLM glm() hot path.

Workload (BASELINE.json configs[1]): binomial/logit GLM on a dense fp64 design of
100M rows x 256 columns per MI355X, resident in HBM, generated on the device by the
seeded synthetic generator (sparkglm_amd.synth; bit-identical host copy).  A "step" is
one IRLS iteration: the fused pass over every resident row (eta, mu, w, z, deviance and
the X'WX / X'Wz Gramian on fp64 MFMA) + the all-reduce over ranks + the p x p solve.

  python bench.py [--gpus N] [--steps K] [--warmup W]
                  [--workload logit256|poisson64|gamma2048|logit512|logit512r|logit1b|lm20]
                  [--rows R] [--p P]

N > 1 runs one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) each process is
one rank; a plain `python bench.py --gpus N` launches those N rank processes itself (through
torch.distributed.run, before anything touches the GPU) and exits with their status.  Each rank
holds its own 100M-row shard (weak scaling) and the per-iteration Gram all-reduce runs on RCCL
over xGMI inside the engine.  Rank 0 prints ONE JSON line.

The default run (N = 1) also measures, after the headline, the north-star 1B x 32 strong point
(`strong_scaling_1b_logit`) and every other BASELINE config's per-GPU shard (`configs_n1`: configs[0]
LM, the configs[2] Poisson, configs[3] gamma and configs[4] procedural shards), each with its own
roofline object; `--no-strong` / `--no-configs` skip them.
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
RIDGE = FP64_MFMA_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)  # ~9.8 flop/B
METRIC = "rows/sec per IRLS iteration + time-to-converge, 1/2/4/8 MI355X"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# BASELINE.json configs -> bench workloads.  The default (N=1 headline) is configs[1]; the others
# are measured in the default run's configs_n1 and with --workload, recorded under profiles/ (rows per GPU = the config's global
# rows / 8 where the config is quoted on 8 GPUs, or the largest resident shard, as labelled).
WORKLOADS = {
    "lm20": dict(cfg=0, kind=1, family="gaussian", link="identity", p=20, rows=1_000_000, seed=1, lm=True,
                 cpu_rows=1_000_000,
                 label="gaussian lm (least squares, LM.fit) on a synthetic 1M x 20 dense design (BASELINE "
                       "configs[0]); a step is one LM fit: Gram pass + solve + residual pass"),
    "logit256": dict(cfg=1, kind=0, family="binomial", link="logit", p=256, rows=100_000_000, seed=2,
                     cpu_rows=2_000_000,
                     label="binomial/logit glm, dense fp64 design, IRLS (BASELINE configs[1])"),
    "poisson64": dict(cfg=2, kind=2, family="poisson", link="log", p=64, rows=125_000_000, seed=3,
                      cpu_rows=8_000_000,
                      label="poisson/log glm with offset + prior weights, 1B x 64 row-sharded over 8 GPUs "
                            "= 125M rows per GPU (BASELINE configs[2])"),
    "gamma2048": dict(cfg=3, kind=3, family="gamma", link="inverse", p=2048, rows=12_500_000, seed=4,
                      cpu_rows=40_000,
                      label="gamma/inverse glm, 50M x 2048 wide design over 4 GPUs = 12.5M rows per GPU, "
                            "GPU Cholesky (BASELINE configs[3])"),
    "logit1b": dict(cfg=1, kind=0, family="binomial", link="logit", p=32, rows=None, strong_rows=1_000_000_000,
                    seed=6, cpu_rows=8_000_000,
                    label="binomial/logit glm, 1B x 32 rows fixed and row-sharded over the N GPUs (north star: "
                          "strong scaling of time-to-convergence on a 1B-row logistic GLM)"),
    "logit512": dict(cfg=4, kind=0, family="binomial", link="logit", p=512, rows=250_000_000, seed=5,
                     cpu_rows=300_000, procedural=True,
                     label="binomial/logit glm, 2B x 512 row-sharded over 8 GPUs = 250M rows per GPU (BASELINE "
                           "configs[4]); 2B x 512 = 8.19 TB exceeds 8 x 288 GB of HBM, so X is procedural: "
                           "regenerated in the pass kernels from the seeded generator, y / eta / w stored"),
    "logit512r": dict(cfg=4, kind=0, family="binomial", link="logit", p=512, rows=60_000_000, seed=5,
                      cpu_rows=300_000,
                      label="binomial/logit glm, p = 512, HBM-resident X: the largest resident shard, 60M rows "
                            "per GPU (BASELINE configs[4] at reduced rows)"),
}


def host_cores(env=None) -> dict:
    """The host cores the CPU baseline runs on ("timed on the same box's host cores,
    with N stated").  N = the cores this process may use: the scheduler affinity mask, capped by
    OMP_NUM_THREADS when the environment sets it -- on the GPU pool every box is a 16-core share
    of a larger host (OMP_NUM_THREADS=16 there; os.cpu_count() reports the whole host's CPUs, which
    this job does not own).  The line records all three numbers."""
    env = os.environ if env is None else env
    total = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = total
    try:
        omp = int(env.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        omp = 0
    threads = max(1, min(affinity, omp) if omp > 0 else affinity)
    return {"threads": threads, "host_cpu_count": total, "affinity_cpus": affinity,
            "omp_num_threads": omp or None}


def cpu_baseline(wl: dict, p: int, rows: int, threads: int | None = None) -> dict:
    """The CPU restatement (oracle/, test infrastructure) timed on a bounded sample, on every host
    core this job owns (host_cores), one Spark-style partition per thread."""
    hc = host_cores()
    threads = threads or hc["threads"]
    res = _cpu_baseline(wl, p, rows, threads)
    res["host_cores"] = hc
    return res


def _cpu_baseline(wl: dict, p: int, rows: int, threads: int) -> dict:
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import pyoracle  # noqa: E402  (checker / CPU baseline only)
    from sparkglm_amd import synth

    X, y, off, prior = synth.generate(wl["kind"], 0, rows, p, wl["seed"])
    if wl.get("lm"):
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            pyoracle.fit_lm(X, y, npart=threads, nthreads=threads)
        dt = (time.perf_counter() - t0) / reps
        return {"value": rows / dt, "unit": "rows/s", "cores": threads, "kind": "port",
                "sample": f"CPU restatement of LM.fit / fitMultiple (oracle/sglm_oracle.c, -O3 AVX2, OpenMP), "
                          f"{rows} x {p} rows of the same generator, {threads} partitions/threads, mean of {reps} "
                          f"fits ({dt * 1e3:.2f} ms each, not the JVM)",
                "time_to_converge_s": dt, "iters": 1}
    t0 = time.perf_counter()
    fit = pyoracle.fit_glm(X, y, wl["family"], wl["link"], offset=off, prior=prior, npart=threads,
                           nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": rows * fit.iter / dt, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": f"CPU restatement of fitMultipleBinomial's IRLS (oracle/sglm_oracle.c, -O3 AVX2, OpenMP), "
                      f"{rows} x {p} {wl['family']}/{wl['link']} rows of the same generator, {threads} "
                      f"partitions/threads, {fit.iter} IRLS iterations to convergence in {dt:.2f} s (not the JVM)",
            "time_to_converge_s": dt, "iters": fit.iter}


def pmc_entry(p: int, family: str, procedural: bool = False):
    """The profiles/pmc_traffic.json entry of a workload shape (rocprofv3 --pmc, tools/pmc_traffic.py)."""
    path = os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            tab = json.load(f)
        key = f"{family}:{p}" + (":proc" if procedural else "")
        return tab.get(key, tab.get(str(p)) if (family == "binomial" and not procedural) else None)
    except (OSError, ValueError):
        return None


def pmc_traffic(p: int, n: int, family: str, procedural: bool = False):
    """Per-launch HBM bytes of the dominant kernel: the per-row FETCH_SIZE + WRITE_SIZE measured
    by rocprofv3 --pmc (profiles/pmc_traffic.json, corrected as MI355X_MICROARCH.md prescribes)
    times the rows of this launch (the pass streams every row exactly once)."""
    e = pmc_entry(p, family, procedural)
    try:
        return None if e is None else e["bytes_per_row"] * n
    except (KeyError, TypeError):
        return None


def lm_traffic(p: int, n: int):
    """(traffic, source) of the LM Gram pass (configs[0]): the stored PMC entry 'gaussian:<p>:lm'
    (tools/pmc_workloads.sh lm20: repeated LM fits, so X -- 168 MB -- comes from the Infinity Cache
    after the first fit; FETCH_SIZE counts L2 fills from the fabric, MALL hits included)."""
    tab = _pmc_table()
    e = tab.get(f"gaussian:{p}:lm")
    if not e or "bytes_per_row" not in e:
        return None, f"none: no PMC pass stored for 'gaussian:{p}:lm'"
    return e["bytes_per_row"] * n, (f"stored PMC, profiles/pmc_traffic.json['gaussian:{p}:lm']: "
                                   f"{e['bytes_per_row']:.2f} B/row measured over {e.get('measured_rows')} rows "
                                   f"({e.get('source', '?')}), x {n} rows of this launch; L2 fills from the fabric "
                                   f"(repeated fits: X from the Infinity Cache)")


def pmc_traffic_source(p: int, n: int, family: str, procedural: bool = False):
    """Where `roofline.traffic` comes from: it is NOT a counter of the timed run but a stored
    rocprofv3 --pmc measurement (bytes per row of a profiling pass over `measured_rows` rows of the
    same shape) scaled to this launch's rows."""
    e = pmc_entry(p, family, procedural)
    if e is None or "bytes_per_row" not in e:
        return None
    key = f"{family}:{p}" + (":proc" if procedural else "")
    tab_key = key if key in _pmc_table() else str(p)
    return (f"stored PMC, profiles/pmc_traffic.json[{tab_key!r}]: {e['bytes_per_row']:.2f} B/row measured over "
            f"{e.get('measured_rows')} rows ({e.get('source', '?')}), x {n} rows of this launch")


def _pmc_table() -> dict:
    try:
        with open(os.path.join(HERE, "profiles", "pmc_traffic.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def mfma_clock_bound(p: int, n: int, family: str, procedural: bool = False) -> dict:
    """The fp64 MFMA instruction stream of a pass -- the second resource of an HBM-bound pass, the
    bound of an MFMA-bound one: the lower-triangular 16x16 tile grid, one v_mfma_f64_16x16x4 per
    tile per 4 rows, 64 cycles on a SIMD, 1024 SIMDs, at the clock the chip held under the kernel
    (PMC GRBM_GUI_ACTIVE), beside the PMC MFMA-busy fraction: where the pass's time goes when it
    is short of its roofline (the power-limited clock, not the 2.4 GHz peak, bounds the stream)."""
    e = pmc_entry(p, family, procedural) or {}
    clk = e.get("clock_ghz")
    t = (p + 15) // 16
    cycles = t * (t + 1) // 2 * (n / 4) * 64 / 1024
    out = {"mfma_tiles": t * (t + 1) // 2, "clock_ghz_pmc": clk, "mfma_busy_frac_pmc": e.get("mfma_busy_frac"),
           "mfma_stream_ms_at_pmc_clock": cycles / (clk * 1e9) * 1e3 if clk else None,
           "mfma_stream_ms_at_2p4ghz": cycles / 2.4e9 * 1e3}
    out.update(fp64_pipe_bound(e, n))
    return out


# Cycles one SIMD spends per wave-instruction on the fp64 pipe (MI355X: 78.6 TF/s fp64 over 1024 SIMDs
# at 2.4 GHz = 32 flop / cycle / SIMD): v_mfma_f64_16x16x4 (2048 flop) 64, an fp64 add / mul / fma
# (64 lanes at 16 lanes a cycle) 4, an fp64 transcendental (quarter rate) 16.
PIPE_CYCLES = {"mfma": 64, "valu": 4, "trans": 16}


def fp64_pipe_bound(e: dict, n: int) -> dict:
    """The fp64 pipe's time for a launch of n rows when the MFMA and the fp64 VALU instructions share
    it: (MFMA cycles + fp64 VALU cycles) / 1024 SIMDs / the PMC clock, from the
    per-row instruction mix the PMC pass measured (profiles/pmc_traffic.json, tools/pmc_workloads.sh
    group 4: SQ_INSTS_VALU_MFMA_F64, SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64).  Empty when the stored
    entry has no mix."""
    clk = e.get("clock_ghz")
    if not clk or "fp64_mfma_insts_per_row" not in e:
        return {}
    per_row = (e["fp64_mfma_insts_per_row"] * PIPE_CYCLES["mfma"] + e["fp64_valu_insts_per_row"] * PIPE_CYCLES["valu"]
               + e.get("fp64_trans_insts_per_row", 0.0) * PIPE_CYCLES["trans"])
    ms = per_row * n / 1024 / (clk * 1e9) * 1e3
    return {"fp64_mfma_insts_per_row": e["fp64_mfma_insts_per_row"],
            "fp64_valu_insts_per_row": e["fp64_valu_insts_per_row"],
            "fp64_trans_insts_per_row": e.get("fp64_trans_insts_per_row", 0.0),
            "pipe_cycles_per_row": per_row, "pipe_bound_ms": ms,
            "pipe_bound_method": "(MFMA x 64 + fp64 VALU x 4 + fp64 transcendental x 16 cycles) / 1024 SIMDs / PMC clock"}


def _free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def needs_launch(env, gpus: int) -> bool:
    """True when this process must spawn the N rank processes itself (no launcher around it)."""
    return gpus > 1 and "WORLD_SIZE" not in env


def launch_cmd(gpus: int, argv, port: int):
    """The torch.distributed.run command of the N ranks (one process per GPU, rendezvous on
    127.0.0.1); every rank re-runs this script with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(gpus: int, argv) -> int:
    """Run the N ranks as child processes (the parent never initialises the GPU) and return the
    first non-zero exit status, else 0.  Rank 0's JSON line reaches stdout unchanged."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    log(f"launching {gpus} rank processes (torch.distributed.run)")
    rc = subprocess.call(launch_cmd(gpus, argv, _free_port()), env=env)
    if rc != 0:
        log(f"rank processes failed with exit status {rc}")
    return rc


# The one JSON line goes here; main() points it at the process's original stdout and sends fd 1
# itself to stderr, so lines that libraries write to stdout (gloo's "[Gloo] Rank 0 is connected
# ..." when ranks rehearse over gloo, runtime banners) cannot come before or into it.
JSON_OUT = sys.stdout


def _guard_stdout() -> None:
    global JSON_OUT
    sys.stdout.flush()
    JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def main() -> int:
    if needs_launch(os.environ, _gpus_arg(sys.argv[1:])):
        return launch_ranks(_gpus_arg(sys.argv[1:]), sys.argv[1:])
    _guard_stdout()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="logit256")
    ap.add_argument("--rows", type=int, default=None, help="rows per GPU (default: the workload's)")
    ap.add_argument("--p", type=int, default=None)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--cpu-rows", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--comm", choices=["rccl", "torch"], default="rccl")
    ap.add_argument("--no-load", action="store_true", help="skip the host-to-HBM load probe")
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the 1B x 32 strong-scaling point measured after the default workload")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the other BASELINE configs' N = 1 points measured after the default workload")
    args = ap.parse_args()
    wl = WORKLOADS[args.workload]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")

    import torch
    import torch.distributed as dist
    from sparkglm_amd import Engine

    dist_on = world > 1
    ndev = max(torch.cuda.device_count(), 1)
    dev = local % ndev  # one rank per GPU; ranks share devices only when rehearsing on fewer GPUs
    # ranks sharing a device (rehearsing N > 1 on fewer GPUs): RCCL refuses duplicate devices,
    # so the group is gloo and the engine all-reduces host buffers through it
    shared = dist_on and world > ndev
    if dist_on:
        torch.cuda.set_device(dev)
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))

    def barrier():
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()

    strong = wl.get("strong_rows") is not None and args.rows is None
    if strong:  # fixed global rows, contiguous shards (Spark's slicing: distributed.shard_range)
        from sparkglm_amd.distributed import shard_range
        lo, hi = shard_range(wl["strong_rows"], world, rank)
        n, row0 = hi - lo, lo
    else:
        n = args.rows or wl["rows"]
        row0 = rank * n
    p = args.p or wl["p"]
    seed = wl["seed"] if args.seed is None else args.seed
    fam, lnk = wl["family"], wl["link"]
    eng = Engine(dev)
    t0 = time.perf_counter()
    eng.synth(wl["kind"], row0, n, p, seed, procedural=wl.get("procedural", False))  # this rank's shard
    gen_s = time.perf_counter() - t0
    attach_comm(eng, args, world, rank, dist_on, shared)
    warm_comm(eng, dist_on, wl["family"], wl["link"])
    log(f"[rank {rank}] shard {n} x {p} ({args.workload}) generated in {gen_s:.2f} s")

    if wl.get("lm"):
        return run_lm(args, wl, eng, n, p, world, rank, dist_on, shared, barrier)

    # time-to-converge: a full fit (data resident), reference semantics (tol 1e-6)
    barrier()
    t0 = time.perf_counter()
    fit = eng.fit_glm(fam, lnk, tol=1e-6)
    barrier()
    ttc = time.perf_counter() - t0
    log(f"[rank {rank}] converged in {fit.iter} iterations, {ttc:.3f} s, deviance {fit.deviance!r}")

    # timed IRLS iterations from the fitted coefficients (a valid eta for every family)
    beta = np.array(fit.coefs, dtype=np.float64)
    if args.warmup > 0:
        beta, _ = eng.irls_iterations(beta, args.warmup, fam, lnk)
    eng.reset_stats()
    barrier()
    t0 = time.perf_counter()
    beta, _ = eng.irls_iterations(beta, args.steps, fam, lnk)
    barrier()
    dt = time.perf_counter() - t0
    st = eng.stats()
    ranks_diag = rank_stats(st, args.steps, dist_on, shared)
    if dist_on:
        tt = torch.tensor([dt, ttc], dtype=torch.float64, device="cpu" if shared else "cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt, ttc = float(tt[0]), float(tt[1])

    if rank == 0:
        total_rows = wl["strong_rows"] if strong else n * world
        passes = max(st["passes"], 1)
        wide = st["path"] == 1
        roof, pass_ms = pass_roofline(st, wl, n, p)
        out = {
            "metric": METRIC,
            "value": total_rows * args.steps / dt,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded counter-based generator, generated in HBM)",
            "config": {"workload": wl["label"], "bench_workload": args.workload,
                       "rows_per_gpu": n, "p": p, "global_rows": total_rows, "parallelism": f"rows{world}" + ("-shared-device-gloo" if shared else ""),
                       "allreduce": "gloo" if shared else ("rccl-engine" if args.comm == "rccl" else "rccl-torch"),
                       "family": fam, "link": lnk, "tol": 1e-6,
                       "offset_prior": wl["kind"] == 2, "procedural_x": wl.get("procedural", False),
                       "comm_warmup": ("one untimed initial-mode pass over the communicator before timing "
                                       "(RCCL peer-connection setup)") if dist_on else None},
            "time_to_converge_s": ttc,
            "iters_to_converge": fit.iter,
            "deviance": fit.deviance,
            "roofline": roof,
            "breakdown_ms_per_step": {"pass_kernels": pass_ms,
                                      "row_kernel": st["row_kernel_ms"] / passes if wide else None,
                                      # wide path: row kernels of chunks >= 1 run beside the Gram on a
                                      # second stream, so row + Gram exceed the pass's wall span
                                      "row_overlap_chunks": st["overlap_chunks"] if wide else None,
                                      "reduce": st["reduce_kernel_ms"] / passes,
                                      "solve": st["solve_ms"] / args.steps,
                                      "comm": st["comm_ms"] / args.steps},
            "ranks": ranks_diag,
            "solve_path": st["solve_path_name"],
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(wl, p, args.cpu_rows or wl["cpu_rows"])
        else:
            out["cpu_baseline"] = None
    eng.close()
    if not args.no_load and rank == 0:
        try:  # the H2D load of a host-resident design, reported apart from the fit;
            # rank 0 only (every rank would otherwise build ~4 GB of host arrays it throws away)
            out["load"] = load_probe(dev, p, wl, n)
        except Exception as exc:
            log(f"[rank {rank}] load probe failed: {exc}")
            out["load"] = None
    if args.workload == "logit256" and not args.no_strong:
        try:  # the north-star 1B-row strong-scaling point, beside the headline (own shard, freed after)
            strong_1b_res = strong_1b(args, dev, world, rank, dist_on, shared, barrier)
        except Exception as exc:  # never lose the headline line to the secondary measurement
            log(f"[rank {rank}] strong-scaling 1B x 32 point failed: {exc}")
            strong_1b_res = None
        if rank == 0:
            out["strong_scaling_1b_logit"] = strong_1b_res
    if args.workload == "logit256" and world == 1 and not args.no_configs:
        out["configs_n1"] = config_points(dev)
    if rank == 0:
        print(json.dumps(out), file=JSON_OUT, flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def pass_roofline(st: dict, wl: dict, n: int, p: int):
    """The `roofline` object of a GLM line (and the pass's wall span in ms) from the engine's stats
    over the timed iterations: the bound follows the pass's arithmetic intensity."""
    fam = wl["family"]
    passes = max(st["passes"], 1)
    wide = st["path"] == 1
    nvec = 1 + (2 if wl["kind"] == 2 else 0)  # y (+ offset, prior)
    flops = n * (p * (p + 1) + 2 * p)      # SYRK-convention X'WX + X'Wz per launch
    bytes_pass = n * (8 * p + 8 * nvec)    # X row + per-row vectors, read once per pass
    # the kernel is the one the engine dispatched (sglm_stats.pass_kernel_name), not re-derived here
    kern = st["pass_kernel_name"] + (" (K1r, split-role fused pass)" if st["pass_kernel_kind"] == "fused-split" else "")
    if wide:
        kern_ms = st["gram_kernel_ms"] / passes
        pass_ms = st["pass_kernel_ms"] / passes  # wall span of the pass (row and Gram may overlap)
    else:
        kern_ms = st["pass_kernel_ms"] / passes
        pass_ms = kern_ms
    tflops = flops / (kern_ms * 1e-3) / 1e12
    gbs = bytes_pass / (pass_ms * 1e-3) / 1e9
    traffic = pmc_traffic(p, n, fam, wl.get("procedural", False))
    traffic_src = pmc_traffic_source(p, n, fam, wl.get("procedural", False))
    if flops / bytes_pass < RIDGE:  # HBM-bound fused pass (arithmetic intensity below the ridge)
        roof = {"bound": "hbm", "kernel": kern, "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": gbs / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                "kernel_ms": kern_ms,
                "algorithmic_bytes_per_launch": bytes_pass,
                "mfma_tflops": tflops, "mfma_frac": tflops / FP64_MFMA_PEAK_TFLOPS,
                "fp64_pipe": mfma_clock_bound(p, n, fam)}
        # how close the pass is to the fp64 pipe's bound, and the HBM fraction that bound allows:
        # an HBM target above it is out of reach at this clock whatever the memory system does
        pb = roof["fp64_pipe"].get("pipe_bound_ms")
        if pb:
            roof["fp64_pipe"]["kernel_frac_of_pipe_bound"] = pb / kern_ms
            roof["fp64_pipe"]["hbm_frac_at_pipe_bound"] = bytes_pass / (pb * 1e-3) / 1e9 / HBM_PEAK_GBS
    else:
        roof = {"bound": "mfma", "kernel": kern, "achieved": tflops, "peak": FP64_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": tflops / FP64_MFMA_PEAK_TFLOPS, "traffic": traffic,
                "traffic_source": traffic_src, "kernel_ms": kern_ms, "algorithmic_flops_per_launch": flops,
                "hbm_gbs_algorithmic": gbs, "fp64_pipe": mfma_clock_bound(p, n, fam, wl.get("procedural", False))}
        # the MFMA instruction stream at the clock the chip holds under the kernel (PMC), against
        # the measured kernel time: how close the kernel is to its clock-limited bound
        sm = roof["fp64_pipe"].get("mfma_stream_ms_at_pmc_clock")
        roof["fp64_pipe"]["kernel_frac_of_clock_limited_stream"] = sm / kern_ms if sm and kern_ms else None
        pb = roof["fp64_pipe"].get("pipe_bound_ms")
        if pb:
            roof["fp64_pipe"]["kernel_frac_of_pipe_bound"] = pb / kern_ms
    return roof, pass_ms


# The other BASELINE configs measured inside the default N = 1 run (after the headline and the strong
# point, each on its own engine, freed before the next), so the driver's run observes every config's
# per-GPU shard, not only builder-side profiles/.  Compact: a fit to convergence, one warm-up
# iteration, CONFIG_STEPS timed iterations (LM: CONFIG_LM_FITS timed fits).
CONFIG_POINTS = ("lm20", "poisson64", "gamma2048", "logit512")
CONFIG_STEPS = 3
CONFIG_LM_FITS = 20


def config_point(name: str, dev: int, rows: int | None = None) -> dict:
    """One BASELINE config's per-GPU shard at N = 1 (the shapes and labels of WORKLOADS): time to
    converge, ms per timed IRLS iteration (LM: per fit), rows/s and the roofline object.  `rows`
    overrides the shard's rows (tests)."""
    import torch
    from sparkglm_amd import Engine
    wl = WORKLOADS[name]
    n, p = rows or wl["rows"], wl["p"]
    eng = Engine(dev)
    try:
        t0 = time.perf_counter()
        eng.synth(wl["kind"], 0, n, p, wl["seed"], procedural=wl.get("procedural", False))
        torch.cuda.synchronize()
        gen_s = time.perf_counter() - t0
        if wl.get("lm"):
            fit = eng.fit_lm()
            eng.reset_stats()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(CONFIG_LM_FITS):
                fit = eng.fit_lm()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / CONFIG_LM_FITS
            st = eng.stats()
            kern_ms = st["pass_kernel_ms"] / max(st["passes"], 1)
            bytes_pass = n * (8 * p + 8)
            gbs = bytes_pass / (kern_ms * 1e-3) / 1e9
            return {"workload": f"{name}: {wl['label']}", "rows": n, "p": p, "generate_s": gen_s,
                    "ms_per_fit": dt * 1e3, "rows_per_s": n / dt, "fits_timed": CONFIG_LM_FITS, "r2": fit.r2,
                    "roofline": {"bound": "hbm", "kernel": st["pass_kernel_name"] + " (LM Gram)", "achieved": gbs,
                                 "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                                 "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": bytes_pass}}
        fam, lnk = wl["family"], wl["link"]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fit = eng.fit_glm(fam, lnk, tol=1e-6)
        torch.cuda.synchronize()
        ttc = time.perf_counter() - t0
        beta = np.array(fit.coefs, dtype=np.float64)
        beta, _ = eng.irls_iterations(beta, 1, fam, lnk)
        eng.reset_stats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.irls_iterations(beta, CONFIG_STEPS, fam, lnk)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / CONFIG_STEPS
        st = eng.stats()
        roof, pass_ms = pass_roofline(st, wl, n, p)
        return {"workload": f"{name}: {wl['label']}", "rows": n, "p": p, "family": fam, "link": lnk,
                "procedural_x": wl.get("procedural", False), "generate_s": gen_s,
                "time_to_converge_s": ttc, "iters_to_converge": fit.iter, "deviance": fit.deviance,
                "ms_per_iter": dt * 1e3, "rows_per_s_per_iter": n / dt, "iters_timed": CONFIG_STEPS,
                "pass_ms": pass_ms, "solve_path": st["solve_path_name"], "roofline": roof}
    finally:
        eng.close()


def config_points(dev: int) -> dict:
    out = {}
    for name in CONFIG_POINTS:
        try:  # never lose the headline line to a secondary measurement
            out[name] = config_point(name, dev)
            log(f"[rank 0] config point {name}: " + (f"{out[name]['ms_per_fit']:.3f} ms per fit" if "ms_per_fit" in out[name]
                                                     else f"{out[name]['ms_per_iter']:.1f} ms per iteration"))
        except Exception as exc:
            log(f"[rank 0] config point {name} failed: {exc}")
            out[name] = {"error": f"{type(exc).__name__}: {exc}"}
    return out


def load_probe(dev: int, p: int, wl: dict, n_shard: int, sample_bytes: float = 4e9) -> dict:
    """Time the ingest boundary on a host-resident sample of the workload's shape: pageable host
    arrays -> sglm_set_data (pinned staging, H2D), as a Spark executor would hand its partitions
    over.  Reported beside the fit, never inside `value` (the fit runs on HBM-resident data)."""
    from sparkglm_amd import Engine
    nvec = 1 + (2 if wl["kind"] == 2 else 0)
    rows = max(1024, int(sample_bytes / (8 * (p + nvec))))
    rng = np.random.default_rng(0)
    X = np.asfortranarray(rng.random((rows, p)))
    y = rng.random(rows)
    vec = (rng.random(rows), rng.random(rows)) if wl["kind"] == 2 else (None, None)
    eng = Engine(dev)
    try:
        eng.set_data(X[:1024], y[:1024])  # first-touch (pinned staging allocation) outside the timing
        eng.reset_stats()
        t0 = time.perf_counter()
        eng.set_data(X, y, offset=vec[0], prior=vec[1])
        wall = time.perf_counter() - t0
        st = eng.stats()
    finally:
        eng.close()
    gbs = st["load_bytes"] / (st["load_ms"] * 1e-3) / 1e9
    shard_bytes = 8.0 * n_shard * (p + nvec)
    return {"sample_rows": rows, "p": p, "bytes": st["load_bytes"], "seconds": st["load_ms"] * 1e-3,
            "wall_seconds": wall, "gbs": gbs, "path": "pageable host -> 2 x 64 MiB pinned staging -> HBM",
            "shard_bytes": shard_bytes, "shard_seconds_est": shard_bytes / (gbs * 1e9) if not wl.get("procedural")
            else None}


def rank_stats(st: dict, iters: int, dist_on: bool, shared: bool) -> dict:
    """Per-rank diagnostics of a multi-GPU line (collective: every rank calls it): pass-kernel,
    reduce-kernel and all-reduce ms per iteration as min and max over the ranks, the all-reduce
    path and whether the scalars went through rank blocks -- enough to tell a compute straggler
    (pass max >> min) from a slow collective (comm) when the scaling curve disappoints."""
    import torch
    import torch.distributed as dist
    it = max(iters, 1)
    v = [st["pass_kernel_ms"] / it, st["reduce_kernel_ms"] / it, st["comm_ms"] / it, st["solve_ms"] / it]
    lo = torch.tensor(v, dtype=torch.float64, device="cpu" if (shared or not dist_on) else "cuda")
    hi = lo.clone()
    if dist_on:
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    lo, hi = lo.cpu().tolist(), hi.cpu().tolist()
    names = ["pass_kernel_ms", "reduce_kernel_ms", "comm_ms", "solve_ms"]
    out = {f"{k}_per_iter_{m}": (a if m == "min" else b) for k, a, b in zip(names, lo, hi) for m in ("min", "max")}
    out["allreduce_path"] = st["comm_path_name"]
    out["scalar_rank_blocks"] = bool(st["rank_blocks"])
    return out


def _gpus_arg(argv) -> int:
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    return ap.parse_known_args(argv)[0].gpus


def attach_comm(eng, args, world: int, rank: int, dist_on: bool, shared: bool) -> None:
    """The engine's per-iteration all-reduce: its own RCCL communicator (sglm_set_comm_rccl),
    else torch's RCCL group, or gloo over host buffers when ranks share a device."""
    import torch
    import torch.distributed as dist
    from sparkglm_amd import Engine
    if shared:
        from sparkglm_amd.distributed import torch_allreduce
        eng.set_comm(torch_allreduce(), on_device=False, rank=rank)
    elif dist_on:
        comm = args.comm
        if comm == "rccl":  # the engine's own RCCL communicator (sglm_set_comm_rccl)
            try:
                uid = [Engine.rccl_unique_id() if rank == 0 else None]
                dist.broadcast_object_list(uid, src=0)
                eng.set_comm_rccl(world, rank, uid[0])
            except Exception as exc:  # same RCCL, reached through torch's process group instead
                log(f"[rank {rank}] engine RCCL communicator unavailable ({exc}); using torch's RCCL group")
                comm = "torch"
            ok = torch.tensor([1 if comm == "rccl" else 0], device="cuda")
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 0:
                comm = "torch"
        if comm != "rccl":
            from sparkglm_amd.distributed import torch_allreduce
            eng.set_comm(torch_allreduce(), on_device=True, rank=rank)
        args.comm = comm


def warm_comm(eng, dist_on: bool, family: str, link: str) -> None:
    """N > 1: one untimed initial-mode pass over the just-attached communicator before anything is
    timed -- a fresh RCCL communicator sets up its peer connections on its first collective, a
    one-time cost of the job (Spark's executors are up before a fit is timed), not of a fit.  The
    pass's results are discarded; every rank makes the same call (collective)."""
    if dist_on:
        eng.irls_pass(None, mu0=0.5, family=family, link=link)


def strong_1b(args, dev: int, world: int, rank: int, dist_on: bool, shared: bool, barrier) -> dict:
    """North-star strong-scaling point measured beside the headline: the 1B x 32 logistic GLM
    (the logit1b workload) row-sharded over the N ranks of this run -- time to converge
    (data resident) and the mean IRLS iteration time, max over ranks."""
    import torch
    import torch.distributed as dist
    from sparkglm_amd import Engine
    from sparkglm_amd.distributed import shard_range
    wl = WORKLOADS["logit1b"]
    lo, hi = shard_range(wl["strong_rows"], world, rank)
    eng = Engine(dev)
    try:
        ok = 1
        try:
            eng.synth(wl["kind"], lo, hi - lo, wl["p"], wl["seed"])
        except Exception as exc:
            log(f"[rank {rank}] 1B x 32 shard not generated: {exc}")
            ok = 0
        if dist_on:  # every rank takes the same branch before any collective of the fit
            f = torch.tensor([ok], device="cpu" if shared else "cuda")
            dist.all_reduce(f, op=dist.ReduceOp.MIN)
            ok = int(f.item())
        if not ok:
            raise RuntimeError("1B x 32 shard not generated on every rank")
        attach_comm(eng, args, world, rank, dist_on, shared)
        warm_comm(eng, dist_on, wl["family"], wl["link"])
        barrier()
        t0 = time.perf_counter()
        fit = eng.fit_glm(wl["family"], wl["link"], tol=1e-6)
        barrier()
        ttc = time.perf_counter() - t0
        beta = np.array(fit.coefs, dtype=np.float64)
        beta, _ = eng.irls_iterations(beta, 1, wl["family"], wl["link"])
        k = 5
        eng.reset_stats()
        barrier()
        t0 = time.perf_counter()
        eng.irls_iterations(beta, k, wl["family"], wl["link"])
        barrier()
        it_s = (time.perf_counter() - t0) / k
        diag = rank_stats(eng.stats(), k, dist_on, shared)
    finally:
        eng.close()
    if dist_on:
        tt = torch.tensor([ttc, it_s], dtype=torch.float64, device="cpu" if shared else "cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        ttc, it_s = float(tt[0]), float(tt[1])
    return {"workload": "logit1b: " + wl["label"], "global_rows": wl["strong_rows"], "p": wl["p"],
            "n_gpus": world, "scaling": "strong", "time_to_converge_s": ttc, "iters_to_converge": fit.iter,
            "deviance": fit.deviance, "ms_per_iter": it_s * 1e3, "rows_per_s_per_iter": wl["strong_rows"] / it_s,
            "ranks": diag}


def run_lm(args, wl, eng, n, p, world, rank, dist_on, shared, barrier) -> int:
    """BASELINE configs[0]: LM.fit (LM.scala:241-274) on the resident shard.  A step is one whole
    fit -- the Gram pass (narrow kernel, LM Gram mode), the all-reduce, the solve and the
    residual pass (rowPartitionedSSE, LM.scala:160-188) -- so rows/s = rows fitted per second."""
    import torch
    import torch.distributed as dist
    fit = eng.fit_lm()
    for _ in range(max(args.warmup, 0)):
        fit = eng.fit_lm()
    eng.reset_stats()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        fit = eng.fit_lm()
    barrier()
    dt = time.perf_counter() - t0
    st = eng.stats()
    if dist_on:
        tt = torch.tensor([dt], dtype=torch.float64, device="cpu" if shared else "cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt[0])
    if rank == 0:
        passes = max(st["passes"], 1)
        kern_ms = st["pass_kernel_ms"] / passes
        bytes_pass = n * (8 * p + 8)  # X row + y, read once by the Gram pass
        gbs = bytes_pass / (kern_ms * 1e-3) / 1e9
        out = {
            "metric": METRIC, "value": n * world * args.steps / dt, "unit": "rows/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded counter-based generator, generated in HBM)",
            "config": {"workload": wl["label"], "bench_workload": args.workload, "rows_per_gpu": n, "p": p,
                       "global_rows": n * world, "parallelism": f"rows{world}", "family": "gaussian (LM)",
                       "link": "identity"},
            "time_to_converge_s": dt / args.steps, "iters_to_converge": 1,
            "r2": fit.r2, "sse": fit.sse,
            "roofline": {"bound": "hbm", "kernel": st["pass_kernel_name"] + " (LM Gram)",
                         "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                         "traffic": lm_traffic(p, n)[0], "traffic_source": lm_traffic(p, n)[1],
                         "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": bytes_pass,
                         "note": "1M x 20 = 168 MB per pass: launch- and latency-bound, not a bandwidth test"},
            "breakdown_ms_per_step": {"gram_pass_kernel": kern_ms, "reduce": st["reduce_kernel_ms"] / args.steps,
                                      "solve": st["solve_ms"] / args.steps, "comm": st["comm_ms"] / args.steps},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(wl, p, args.cpu_rows or wl["cpu_rows"])
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), file=JSON_OUT, flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()
    return 0


def _run() -> int:
    """main() with a named failure: a rank whose fit fails (e.g. SGLM_ECOMM when a peer rank died
    and the all-reduce missed its SGLM_COMM_TIMEOUT_S deadline) says which rank and why and exits
    non-zero at once, without waiting in a collective of the torch group for peers that are gone."""
    try:
        return main()
    except Exception as exc:  # noqa: BLE001  (reported, then a non-zero exit)
        import traceback
        traceback.print_exc(file=sys.stderr)
        log(f"[rank {os.environ.get('RANK', '0')}] bench failed: {type(exc).__name__}: {exc}")
        sys.stderr.flush()
        os._exit(1)


if __name__ == "__main__":
    sys.exit(_run())
