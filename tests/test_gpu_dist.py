"""Multi-rank GPU paths on one MI355X: rank processes sharing the device with the engine's
host all-reduce over gloo, the native RCCL communicator, torch's RCCL ("nccl") group through
the device-buffer callback -- and, at world 2 and 4, the DEVICE-buffer all-reduce path
(stage_rank_block + the rank blocks of the packed buffer in HBM, engine.cpp) over a gloo group
of CUDA tensors: the buffers and the staging an RCCL communicator carries across GPUs, exercised
with several ranks before an 8-GPU node runs them (utils.scala:110-126, GLM.scala:404-407)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, rel

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, mode, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from sparkglm_amd import Engine, synth
    from sparkglm_amd import distributed as D
    n_global, p = 40_000, 48
    lo, hi = D.shard_range(n_global, world, rank)
    X, y, off, pr = synth.generate(2, lo, hi - lo, p, 5)
    eng = Engine(0)
    eng.set_data(X, y, offset=off, prior=pr)
    if mode == "gloo":
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        eng.set_comm(D.torch_allreduce(), on_device=False, rank=rank)
    elif mode == "rccl":
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        uid = [Engine.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.set_comm_rccl(world, rank, uid[0])
    elif mode == "gloo-device":  # device buffers through a gloo group of CUDA tensors
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        eng.set_comm(D.torch_allreduce(), on_device=True, rank=rank)
    else:  # torch nccl group, device buffers
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        eng.set_comm(D.torch_allreduce(), on_device=True, rank=rank)
    f = eng.fit_glm("poisson", "log", init="multiple")
    st = eng.stats()
    q.put((rank, (f.coefs, f.stderr, np.array([f.deviance, f.null_deviance, f.pearson, f.loglik, f.iter, f.nrow,
                                                f.npart]), (st["comm_path_name"], st["rank_blocks"]))))
    dist.barrier()
    eng.close()
    dist.destroy_process_group()


def _run(mode, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def _reference(world):
    """fitMultipleBinomial over `world` row partitions (the partitioned oracle)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    from sparkglm_amd import synth
    X, y, off, pr = synth.generate(2, 0, 40_000, 48, 5)
    return po.fit_glm(X, y, "poisson", "log", offset=off, prior=pr, npart=max(world, 2), nthreads=2)


PATH = {"gloo": "caller-host", "gloo-device": "caller-device", "rccl": "rccl", "nccl": "caller-device"}


@pytest.mark.parametrize("mode,world", [("gloo", 2), ("rccl", 1), ("nccl", 1), ("gloo-device", 2),
                                        ("gloo-device", 4)])
def test_sharded_fit_equals_oracle(mode, world):
    res = _run(mode, world)
    ref = _reference(world)
    for r in range(world):
        coefs, se, s, (path, blocks) = res[r]
        assert path == PATH[mode], path
        assert blocks == (1 if world > 1 else 0)  # the scalars through the rank blocks of the buffer
        assert int(s[4]) == ref.iter and s[5] == 40_000 and int(s[6]) == world
        assert rel(coefs, ref.coefs) < 1e-9 and rel(se, ref.stderr) < 1e-9
        assert rel(s[:4], [ref.deviance, ref.null_deviance, ref.pearson, ref.loglik]) < 1e-9


def _fail_worker(rank, world, port, case, q):
    """Failure modes of the rank protocol: `badrank` -- rank 1 passes an out-of-range rank to
    sglm_set_comm_rank (every rank must still join the check's all-reduce and all of them
    get SGLM_EINVAL); `deadpeer` -- rank 1 exits before the fit's first collective, rank 0 must get
    SGLM_ECOMM within SGLM_COMM_TIMEOUT_S instead of hanging."""
    sys.path.insert(0, ROOT)
    os.environ["SGLM_COMM_TIMEOUT_S"] = "10"
    import time
    import torch
    import torch.distributed as dist
    from sparkglm_amd import Engine, synth
    from sparkglm_amd import distributed as D
    from sparkglm_amd._lib import CommError, IllegalArgumentException
    X, y, off, pr = synth.generate(2, 1000 * rank, 1000, 8, 5)
    eng = Engine(0)
    eng.set_data(X, y, offset=off, prior=pr)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    if case == "badrank":
        try:
            eng.set_comm(D.torch_allreduce(), on_device=True, rank=5 if rank == 1 else rank)
            q.put((rank, "no error"))
        except IllegalArgumentException as exc:
            q.put((rank, "einval:" + str(exc)))
        dist.barrier()
        eng.close()
        dist.destroy_process_group()
        return
    eng.set_comm(D.torch_allreduce(), on_device=True, rank=rank)

    def put_and_exit(item):
        # os._exit skips the queue's feeder thread: flush the item to the pipe first
        q.put(item)
        q.close()
        q.join_thread()
        os._exit(0)

    if rank == 1:
        put_and_exit((rank, "exited"))  # dies before the fit's first collective
    t0 = time.perf_counter()
    try:
        eng.fit_glm("poisson", "log", init="multiple")
        item = (rank, "no error")
    except CommError as exc:
        item = (rank, f"ecomm:{time.perf_counter() - t0:.1f}:{exc}")
    put_and_exit(item)  # the gloo group lost a member: skip its teardown


@pytest.mark.parametrize("case", ["badrank", "deadpeer"])
def test_rank_failures_end_with_an_error_not_a_hang(case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=150) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    if case == "badrank":
        for r in (0, 1):
            assert res[r].startswith("einval:") and "distinct rank" in res[r], res[r]
    else:
        assert res[1] == "exited"
        assert res[0].startswith("ecomm:"), res[0]
        assert float(res[0].split(":")[1]) < 60.0, res[0]


def test_rccl_deadline_counts_from_the_end_of_the_pass(monkeypatch):
    """the RCCL all-reduce's deadline starts when this rank's own pass has
    finished (wait_collective polls the pass-end event first), so a pass longer than
    SGLM_COMM_TIMEOUT_S on a large shard does not abort a healthy communicator.  World 1 over the
    engine's RCCL communicator, a 50 ms deadline against the ~110 ms passes of configs[1]'s 100M x 256
    shard: the fit completes over RCCL and matches the streaming oracle's full-size fit."""
    import json
    from sparkglm_amd import Engine
    fs = os.path.join(ROOT, "tests", "golden", "full_scale.json")
    if not os.path.exists(fs):
        pytest.skip("full_scale.json absent")
    c = json.load(open(fs))["logit256"]
    monkeypatch.setenv("SGLM_COMM_TIMEOUT_S", "0.05")
    with Engine(0) as e:
        e.synth(c["kind"], c["row0"], c["n"], c["p"], c["seed"])
        e.set_comm_rccl(1, 0, Engine.rccl_unique_id())
        f = e.fit_glm(c["family"], c["link"], tol=c["tol"])
        st = e.stats()
    assert st["comm_path_name"] == "rccl" and st["pass_kernel_ms"] / max(st["passes"], 1) > 60.0
    assert f.iter == c["iter"]
    assert rel(f.coefs, c["coefs"]) < 1e-9 and rel(f.stderr, c["stderr"]) < 1e-9
    assert rel(f.deviance, c["deviance"]) < 1e-9
