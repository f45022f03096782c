"""bench.py's contract pieces: every workload maps to a BASELINE.json config with the family /
shape it names, the traffic lookup, and the roofline bound choice (no GPU); the default run's
config points on the device (gpu)."""
import importlib.util
import json
import os

import pytest

from conftest import ROOT

spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)


def test_workloads_follow_baseline_configs():
    cfgs = json.load(open(os.path.join(ROOT, "BASELINE.json")))["configs"]
    assert bench.WORKLOADS["logit256"]["cfg"] == 1  # the default = the headline config
    for name, wl in bench.WORKLOADS.items():
        text = cfgs[wl["cfg"]].lower()
        fam = wl["family"].lower()
        assert fam in text or (fam == "binomial" and "logit" in text), name
        if wl.get("strong_rows") is None:
            assert str(wl["p"]) in text.replace("×", "x"), name
    assert bench.WORKLOADS["logit512"]["procedural"] is True  # 2B x 512 cannot be resident
    assert bench.WORKLOADS["logit1b"]["strong_rows"] == 1_000_000_000


def test_roofline_bound_follows_arithmetic_intensity():
    # flops p(p+1)+2p, bytes 8p + 8k per row; ridge = 78.6 TF / 8 TB/s
    def bound(p, nvec):
        return "hbm" if (p * (p + 1) + 2 * p) / (8 * p + 8 * nvec) < bench.RIDGE else "mfma"
    assert bound(64, 3) == "hbm" and bound(32, 1) == "hbm"
    assert bound(256, 1) == "mfma" and bound(512, 1) == "mfma" and bound(2048, 1) == "mfma"


def test_pmc_traffic_lookup():
    t = bench.pmc_traffic(256, 1000, "binomial")
    assert t is not None and 2000 * 1000 < t < 2200 * 1000
    # the procedural shard has its own entry (its scratch writes are part of its traffic)
    import json as _json
    tab = _json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    assert bench.pmc_traffic(512, 10, "binomial", procedural=True) == tab["binomial:512:proc"]["bytes_per_row"] * 10
    assert bench.pmc_traffic(512, 10, "binomial") == tab["binomial:512"]["bytes_per_row"] * 10
    assert bench.pmc_traffic(333, 10, "binomial") is None


def test_roofline_traffic_is_the_stored_pmc_scaled_and_says_so():
    # the line's `traffic` is the stored PMC bytes/row x the launch's rows, and
    # `traffic_source` names the table entry and its profiling size
    tab = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    for name, wl in bench.WORKLOADS.items():
        if wl.get("lm"):
            continue
        n = wl["rows"] or wl["strong_rows"]
        proc = wl.get("procedural", False)
        key = f"{wl['family']}:{wl['p']}" + (":proc" if proc else "")
        t = bench.pmc_traffic(wl["p"], n, wl["family"], proc)
        src = bench.pmc_traffic_source(wl["p"], n, wl["family"], proc)
        assert key in tab, name
        assert t == tab[key]["bytes_per_row"] * n, name
        assert src.startswith("stored PMC, profiles/pmc_traffic.json") and repr(key) in src, name
        assert str(tab[key]["measured_rows"]) in src and f"x {n} rows" in src, name
    assert bench.pmc_traffic_source(333, 10, "binomial") is None


def test_every_baseline_config_has_a_workload():
    cfgs = json.load(open(os.path.join(ROOT, "BASELINE.json")))["configs"]
    assert {wl["cfg"] for wl in bench.WORKLOADS.values()} == set(range(len(cfgs)))
    assert bench.WORKLOADS["lm20"]["cfg"] == 0 and bench.WORKLOADS["lm20"].get("lm")


def test_strong_scaling_point_and_p32_traffic():
    # the default run appends the north-star 1B x 32 strong-scaling point (bench.strong_1b),
    # whose per-row PMC traffic the logit1b roofline uses
    assert callable(bench.strong_1b) and callable(bench.attach_comm)
    t = bench.pmc_traffic(32, 1000, "binomial")
    assert t is not None and 264 * 1000 <= t < 280 * 1000


def test_plain_multi_gpu_invocation_launches_its_own_ranks():
    """`python bench.py --gpus N` without a launcher spawns N rank processes (torch.distributed.run,
    rendezvous on 127.0.0.1) running this script with the same arguments; under a launcher
    (WORLD_SIZE set) or at N = 1 it runs in-process."""
    assert bench.needs_launch({}, 2) and bench.needs_launch({"RANK": "0"}, 8)
    assert not bench.needs_launch({"WORLD_SIZE": "2"}, 2) and not bench.needs_launch({}, 1)
    assert bench._gpus_arg(["--steps", "3", "--gpus", "4"]) == 4 and bench._gpus_arg([]) == 1
    argv = ["--gpus", "4", "--steps", "3", "--warmup", "1"]
    cmd = bench.launch_cmd(4, argv, 29511)
    i = cmd.index("torch.distributed.run")
    assert cmd[i - 1] == "-m" and "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert "--master-port=29511" in cmd and "--nnodes=1" in cmd
    assert cmd[-len(argv) - 1].endswith("bench.py") and cmd[-len(argv):] == argv


def test_launcher_runs_ranks_with_rank_environment(tmp_path):
    """The launch path end to end on CPU: torch.distributed.run gives every child the RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* environment bench.py's rank code reads."""
    import subprocess
    import sys
    probe = tmp_path / "probe.py"
    # one file per rank: two ranks printing to one pipe can interleave their lines
    probe.write_text("import os, json\nd = {k: os.environ.get(k) for k in ('RANK','LOCAL_RANK','WORLD_SIZE','MASTER_ADDR')}\n"
                     f"open(os.path.join({str(tmp_path)!r}, 'rank' + d['RANK'] + '.json'), 'w').write(json.dumps(d))\n")
    cmd = bench.launch_cmd(2, [], bench._free_port())
    cmd[cmd.index(os.path.abspath(bench.__file__))] = str(probe)
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    envs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in (0, 1)]
    assert sorted(e["RANK"] for e in envs) == ["0", "1"]
    assert all(e["WORLD_SIZE"] == "2" and e["MASTER_ADDR"] == "127.0.0.1" for e in envs)


def test_stdout_carries_only_the_json_line():
    """Rank processes send fd 1 to stderr (gloo and runtimes print there) and keep the original
    stdout for the one JSON line the driver parses."""
    import subprocess
    import sys
    code = ("import os, sys, json; sys.path.insert(0, %r); import bench; bench._guard_stdout(); "
            "os.write(1, b'[Gloo] Rank 0 is connected to 1 peer ranks.\\n'); print('log line'); "
            "print(json.dumps({'metric': 'm'}), file=bench.JSON_OUT, flush=True)") % os.path.dirname(bench.__file__)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.splitlines() == ['{"metric": "m"}']
    assert "[Gloo]" in out.stderr and "log line" in out.stderr


def _rank_stats_worker(rank, world, port, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    st = {"pass_kernel_ms": 100.0 + 10 * rank, "reduce_kernel_ms": 1.0, "comm_ms": 5.0 * (rank + 1),
          "solve_ms": 2.0, "comm_path_name": "caller-host", "rank_blocks": 1}
    q.put((rank, bench.rank_stats(st, 10, True, True)))
    dist.barrier()
    dist.destroy_process_group()


def test_rank_diagnostics_field_layout():
    """the multi-GPU lines carry per-rank pass-kernel / reduce / all-reduce /
    solve ms per iteration as min and max over the ranks, the all-reduce path and whether the
    scalars crossed the ranks in rank blocks -- on one process and over a gloo world of 2."""
    st = {"pass_kernel_ms": 50.0, "reduce_kernel_ms": 0.5, "comm_ms": 0.0, "solve_ms": 1.0,
          "comm_path_name": "none", "rank_blocks": 0}
    d = bench.rank_stats(st, 5, False, False)
    assert d["pass_kernel_ms_per_iter_min"] == d["pass_kernel_ms_per_iter_max"] == 10.0
    assert d["allreduce_path"] == "none" and d["scalar_rank_blocks"] is False
    assert set(d) == {f"{k}_per_iter_{m}" for k in ("pass_kernel_ms", "reduce_kernel_ms", "comm_ms", "solve_ms")
                      for m in ("min", "max")} | {"allreduce_path", "scalar_rank_blocks"}
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench._free_port()
    ps = [ctx.Process(target=_rank_stats_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        assert res[r]["pass_kernel_ms_per_iter_min"] == 10.0 and res[r]["pass_kernel_ms_per_iter_max"] == 11.0
        assert res[r]["comm_ms_per_iter_min"] == 0.5 and res[r]["comm_ms_per_iter_max"] == 1.0
        assert res[r]["allreduce_path"] == "caller-host" and res[r]["scalar_rank_blocks"] is True


def test_mfma_clock_bound_counts_the_tile_stream():
    # one v_mfma_f64_16x16x4 per lower-triangular 16x16 tile per 4 rows, 64 cycles on one of 1024
    # SIMDs, at the PMC clock of the workload shape (profiles/pmc_traffic.json)
    e = bench.mfma_clock_bound(256, 100_000_000, "binomial")
    assert e["mfma_tiles"] == 136
    clk = bench.pmc_entry(256, "binomial")["clock_ghz"]
    cycles = 136 * 25_000_000 * 64 / 1024
    assert abs(e["mfma_stream_ms_at_pmc_clock"] - cycles / (clk * 1e9) * 1e3) < 1e-9
    assert abs(e["mfma_stream_ms_at_2p4ghz"] - cycles / 2.4e9 * 1e3) < 1e-9
    assert bench.mfma_clock_bound(2048, 10, "gamma")["mfma_tiles"] == 128 * 129 // 2
    # the procedural shard has its own PMC entry (clock under the generator + Gram)
    assert bench.mfma_clock_bound(512, 10, "binomial", True)["clock_ghz_pmc"] == \
        bench.pmc_entry(512, "binomial", True)["clock_ghz"]


def test_pmc_traffic_counts_every_dispatch_of_a_pass(tmp_path, monkeypatch):
    # tools/pmc_traffic.py: a chunked wide pass dispatches its Gram kernels once per chunk; the
    # per-row bytes sum every dispatch and divide by the passes (one chunk-0 row kernel each)
    spec2 = importlib.util.spec_from_file_location("pmc_traffic", os.path.join(ROOT, "tools", "pmc_traffic.py"))
    pt = importlib.util.module_from_spec(spec2)
    spec2.loader.exec_module(pt)
    rows = pt.WL["gamma2048"][1]
    fake = {  # per-dispatch averages (FETCH_SIZE in KB: half of the streamed bytes on gfx950)
        "void sglm::wide_rows_kernel<3, 5>(sglm::WideRowArgs)": {"FETCH_SIZE": 100.0, "WRITE_SIZE": 0.0, "dispatches": 2,
                                                                "avg_ms": 1.0, "GRBM_GUI_ACTIVE": 8e6,
                                                                "SQ_VALU_MFMA_BUSY_CYCLES": 0.0},
        "void sglm::wide_gram_kernel<false, false>(sglm::WideGramArgs)": {"FETCH_SIZE": 1000.0, "WRITE_SIZE": 1.0,
                                                                         "dispatches": 6, "avg_ms": 10.0,
                                                                         "GRBM_GUI_ACTIVE": 8e7,
                                                                         "SQ_VALU_MFMA_BUSY_CYCLES": 1e9},
    }
    monkeypatch.setattr(pt, "load", lambda d, wl: fake)
    (tmp_path / "gamma2048_1").mkdir()
    out = tmp_path / "t.json"
    monkeypatch.setattr(pt.sys, "argv", ["pmc_traffic.py", str(tmp_path), "test", str(out)])
    pt.main()
    e = json.load(open(out))["gamma:2048"]
    per_pass_kb = 100.0 * 2 / 2 + 1000.0 * 6 / 2      # 2 passes: 1 row + 3 Gram dispatches each
    assert abs(e["fetch_bytes_per_row"] - per_pass_kb * 2 * 1024 / rows) < 1e-9
    assert abs(e["write_bytes_per_row"] - 1.0 * 6 / 2 * 1024 / rows) < 1e-9
    assert abs(e["kernel_ms_profiled"] - (1.0 + 30.0)) < 1e-12


def test_fp64_pipe_bound_reproduces_from_the_stored_pmc_mix():
    # an HBM-bound line carries the fp64 pipe's bound -- (MFMA x 64 + fp64 VALU x 4
    # + transcendental x 16 cycles) / 1024 SIMDs / PMC clock -- from profiles/pmc_traffic.json's
    # instruction mix, so kernel_frac_of_pipe_bound reproduces from profiles/
    e = bench.pmc_entry(64, "poisson")
    assert e["fp64_mfma_insts_per_row"] == 2.5  # 10 lower-triangular 16x16 tiles per 4 rows: the counter's scale
    b = bench.mfma_clock_bound(64, 125_000_000, "poisson")
    cyc = 2.5 * 64 + e["fp64_valu_insts_per_row"] * 4 + e["fp64_trans_insts_per_row"] * 16
    assert abs(b["pipe_cycles_per_row"] - cyc) < 1e-9
    assert abs(b["pipe_bound_ms"] - cyc * 125_000_000 / 1024 / (e["clock_ghz"] * 1e9) * 1e3) < 1e-9
    # at p = 64 the pipe bound sits below the 70 % HBM target: 536 B / row at the bound < 0.7 x 8 TB/s
    hbm_frac = 125_000_000 * 536 / (b["pipe_bound_ms"] * 1e-3) / 1e9 / bench.HBM_PEAK_GBS
    assert 0.55 < hbm_frac < 0.70
    assert bench.fp64_pipe_bound({"clock_ghz": 2.0}, 10) == {}  # no stored mix: no bound claimed


def test_cpu_baseline_states_its_cores():
    # the CPU baseline runs on every host core the job owns -- the affinity mask,
    # capped by OMP_NUM_THREADS when set (the GPU pool's 16-core share) -- and says so
    import os as _os
    aff = len(_os.sched_getaffinity(0))
    hc = bench.host_cores({"OMP_NUM_THREADS": "4"})
    assert hc["threads"] == min(4, aff) and hc["affinity_cpus"] == aff and hc["omp_num_threads"] == 4
    assert hc["host_cpu_count"] == (_os.cpu_count() or 1)
    assert bench.host_cores({})["threads"] == aff and bench.host_cores({})["omp_num_threads"] is None
    assert bench.host_cores({"OMP_NUM_THREADS": "junk"})["threads"] == aff


def test_lm_line_traffic_comes_from_the_lm_pmc_entry():
    # the lm20 line's roofline.traffic was null; now the stored PMC of the LM Gram
    # pass (tools/pmc_workloads.sh lm20 -> pmc_traffic.json['gaussian:20:lm'])
    tab = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    t, src = bench.lm_traffic(20, 1_000_000)
    assert t == tab["gaussian:20:lm"]["bytes_per_row"] * 1_000_000
    assert "gaussian:20:lm" in src and "Infinity Cache" in src
    assert bench.lm_traffic(7, 10)[0] is None


def test_default_run_covers_every_baseline_config():
    # the headline (configs[1]) + the strong 1B point + configs_n1: every config's per-GPU shard is
    # measured by the driver's own default run, not only by builder-side --workload runs
    cfgs = json.load(open(os.path.join(ROOT, "BASELINE.json")))["configs"]
    covered = {bench.WORKLOADS["logit256"]["cfg"]} | {bench.WORKLOADS[w]["cfg"] for w in bench.CONFIG_POINTS}
    assert covered == set(range(len(cfgs)))
    assert "logit256" not in bench.CONFIG_POINTS and bench.CONFIG_STEPS >= 1


def test_pass_roofline_from_stats():
    # a fused-pass line: the kernel time is the pass time; MFMA-bound at p = 256
    st = {"passes": 2, "path": 0, "pass_kernel_name": "k", "pass_kernel_kind": "fused-split",
          "pass_kernel_ms": 200.0, "gram_kernel_ms": 0.0}
    roof, pass_ms = bench.pass_roofline(st, bench.WORKLOADS["logit256"], 100_000_000, 256)
    assert roof["bound"] == "mfma" and pass_ms == 100.0 and roof["kernel_ms"] == 100.0
    assert abs(roof["achieved"] - 1e8 * (256 * 257 + 512) / 0.1 / 1e12) < 1e-9
    # a wide line: the Gram kernels are the dominant kernel, the pass span is the wall clock
    st = dict(st, path=1, pass_kernel_kind="wide", pass_kernel_ms=600.0, gram_kernel_ms=560.0)
    roof, pass_ms = bench.pass_roofline(st, bench.WORKLOADS["gamma2048"], 12_500_000, 2048)
    assert roof["bound"] == "mfma" and pass_ms == 300.0 and roof["kernel_ms"] == 280.0
    # an HBM-bound narrow line carries the fp64-pipe fractions
    st = dict(st, path=0, pass_kernel_kind="narrow", pass_kernel_ms=28.0)
    roof, _ = bench.pass_roofline(st, bench.WORKLOADS["poisson64"], 125_000_000, 64)
    assert roof["bound"] == "hbm" and roof["unit"] == "GB/s"
    assert "kernel_frac_of_pipe_bound" in roof["fp64_pipe"]


@pytest.mark.gpu
@pytest.mark.parametrize("name,rows", [("lm20", 200_000), ("poisson64", 400_000), ("gamma2048", 20_000),
                                       ("logit512", 100_000)])
def test_config_point_runs_on_the_device(name, rows):
    """The default bench run's configs_n1 points (bench.config_point) at reduced rows: each fits,
    times its iterations and carries a roofline object with the bound SURVEY 8(d) assigns."""
    r = bench.config_point(name, 0, rows=rows)
    assert r["rows"] == rows and r["p"] == bench.WORKLOADS[name]["p"]
    roof = r["roofline"]
    assert roof["frac"] > 0 and roof["kernel_ms"] > 0
    if name == "lm20":
        assert r["ms_per_fit"] > 0 and roof["bound"] == "hbm"
    else:
        assert r["iters_to_converge"] >= 1 and r["ms_per_iter"] > 0
        assert roof["bound"] == ("hbm" if name == "poisson64" else "mfma")
        assert r["procedural_x"] == (name == "logit512")
