"""Multi-rank path on CPU: world_size 2 over gloo.  Each rank holds its row shard; the
engine's C++ driver runs on every rank and all-reduces the packed partials through the
torch.distributed communicator adapter -- the same protocol a GPU rank uses.  Partials
come from the oracle here (CPU host, checker), results must equal the single-process fit."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, rel


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, case, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist
    import pyoracle as po
    from sparkglm_amd import distributed as D
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    X, y, fam, link, kw = case
    lo, hi = D.shard_range(len(y), world, rank)
    Xs, ys = np.asfortranarray(X[lo:hi]), y[lo:hi]
    kws = {k: (None if v is None else v[lo:hi]) for k, v in kw.items()}
    sums = lambda: (ys.sum(), len(ys))
    if fam == "lm":
        part = lambda mode, b, mu0, ybar: po.shard_partials(Xs, ys, "gaussian", "identity", mode, b, mu0, ybar)
        f = D.fit_lm_external(X.shape[1], sums, part, allreduce=D.torch_allreduce())
        out = (f.coefs, f.stderr, np.array([f.sse, f.r2, f.fstat, f.nrow, f.npart]))
    else:
        part = lambda mode, b, mu0, ybar: po.shard_partials(Xs, ys, fam, link, mode, b, mu0, ybar, **kws)
        f = D.fit_glm_external(X.shape[1], sums, part, allreduce=D.torch_allreduce(), family=fam, link=link,
                               init="multiple")
        out = (f.coefs, f.stderr, np.array([f.deviance, f.null_deviance, f.pearson, f.loglik, f.iter, f.nrow,
                                            f.npart]))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def _run(case, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_shard_range_partitions_rows():
    from sparkglm_amd.distributed import shard_range
    for n in (0, 1, 7, 100, 101):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))


@pytest.mark.parametrize("name", ["logit", "poisson_offset_prior"])
def test_gloo_two_ranks_glm_equals_single_process(golden, name):
    import pyoracle as po
    c = golden[name]
    fam, link = (str(v) for v in c["meta"][:2])
    kw = {"offset": c.get("offset"), "prior": c.get("prior"), "m": c.get("m")}
    res = _run((c["X"], c["y"], fam, link, kw))
    ref = po.fit_glm(c["X"], c["y"], fam, link, npart=2, nthreads=2, **kw)
    for r in (0, 1):
        coefs, se, s = res[r]
        assert int(s[4]) == ref.iter and int(s[6]) == 2 and s[5] == len(c["y"])
        assert rel(coefs, ref.coefs) < 1e-10 and rel(se, ref.stderr) < 1e-10
        assert rel(s[:4], [ref.deviance, ref.null_deviance, ref.pearson, ref.loglik]) < 1e-10
    np.testing.assert_array_equal(res[0][0], res[1][0])  # every rank holds the same fit


def test_gloo_two_ranks_lm_equals_single_process(golden):
    import pyoracle as po
    c = golden["gaussian"]
    res = _run((c["X"], c["y"], "lm", None, {}))
    ref = po.fit_lm(c["X"], c["y"])
    for r in (0, 1):
        coefs, se, s = res[r]
        assert rel(coefs, ref["coefs"]) < 1e-10 and rel(se, ref["stderr"]) < 1e-10
        assert rel(s[:3], [ref["sse"], ref["r2"], ref["fstat"]]) < 1e-10
