"""First-contact check of the split-role narrow pass (narrow_r.hip) on a GPU: small fits through
irls_narrow_r_kernel against the same fits through irls_narrow_kernel (SGLM_NARROW_SPLIT=0), then
the pass time of both on a bench-sized shard.  Development tool (the parity tests are
tests/test_gpu_narrow_split.py)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sparkglm_amd import Engine  # noqa: E402


def engine(split):
    os.environ["SGLM_NARROW_SPLIT"] = str(split)
    try:
        return Engine(0)
    finally:
        os.environ.pop("SGLM_NARROW_SPLIT", None)


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))


def fit_pair(kind, n, p, fam, lnk, split):
    out = []
    for s in (split, 0):
        e = engine(s)
        e.synth(kind, 0, n, p, 7)
        f = e.fit_glm(fam, lnk, init="multiple")
        st = e.stats()
        out.append((f, st["pass_kernel_name"]))
        e.close()
    (a, ka), (b, kb) = out
    print(f"{fam}/{lnk} n={n} p={p}: {ka} vs {kb}: iter {a.iter}/{b.iter} dev rel {rel(a.deviance, b.deviance):.2e} "
          f"coef rel {rel(a.coefs, b.coefs):.2e} se rel {rel(a.stderr, b.stderr):.2e} "
          f"pearson {rel(a.pearson, b.pearson):.2e} ll {rel(a.loglik, b.loglik):.2e}", flush=True)
    assert a.iter == b.iter and rel(a.deviance, b.deviance) < 1e-11 and rel(a.coefs, b.coefs) < 1e-9
    assert "narrow_r" in ka and "narrow_r" not in kb


def lm_pair(n, p, split):
    out = []
    for s in (split, 0):
        e = engine(s)
        e.synth(1, 0, n, p, 3)
        out.append((e.fit_lm(), e.stats()["pass_kernel_name"]))
        e.close()
    (a, ka), (b, kb) = out
    print(f"LM n={n} p={p}: {ka} vs {kb}: coef rel {rel(a.coefs, b.coefs):.2e} sse rel {rel(a.sse, b.sse):.2e}", flush=True)
    assert rel(a.coefs, b.coefs) < 1e-9


def timing(kind, n, p, fam, lnk, passes=5):
    b = np.full(p, 0.01)
    for s in (3, 0, 3, 0):
        e = engine(s)
        e.synth(kind, 0, n, p, 2)
        e.irls_pass(b, family=fam, link=lnk)
        e.reset_stats()
        for _ in range(passes):
            e.irls_pass(b, family=fam, link=lnk)
        st = e.stats()
        print(f"timing {fam} n={n} p={p} split={s}: {st['pass_kernel_name']} {st['pass_kernel_ms'] / st['passes']:.3f} ms/pass",
              flush=True)
        e.close()


if __name__ == "__main__":
    stage = sys.argv[1] if len(sys.argv) > 1 else "all"
    t0 = time.time()
    if stage in ("all", "parity"):
        n = 32 * 9377 - 5  # odd 32-row block count: the short last 64-row block
        fit_pair(2, n, 64, "poisson", "log", 3)
        fit_pair(2, n, 40, "poisson", "log", 3)
        fit_pair(0, n, 64, "binomial", "logit", 3)
        fit_pair(0, n, 48, "binomial", "probit", 3)
        fit_pair(3, n, 64, "gamma", "inverse", 3)
        fit_pair(0, n, 32, "binomial", "logit", 2)
        fit_pair(0, 1000, 64, "binomial", "logit", 3)   # fewer blocks than workgroups
        lm_pair(1_000_000, 40, 3)
        lm_pair(1_000_000, 20, 2)
        print(f"parity ok ({time.time() - t0:.1f} s)", flush=True)
    if stage in ("all", "timing"):
        timing(2, 125_000_000, 64, "poisson", "log")
        timing(0, 200_000_000, 32, "binomial", "logit") if os.environ.get("NR_P32") else None
