"""Full-scale golden fits of the bench workloads, from the streaming oracle.

SURVEY.md 8(d): parity at the sizes the bench runs, rows regenerated on the fly from the
same seeded generator (oracle/sglm_oracle.c `orc_fit_glm_synth`; the generator is
bit-identical to sparkglm_amd.synth and to the device's sglm_synth).  Run once in the CPU
container (about 20 minutes on 8 cores); the GPU test tests/test_gpu_full_scale.py fits
the same shards in HBM and compares coefficients / standard errors / deviance at 1e-9 with
the same iteration count, printing the final |delta deviance| beside tol.

    python tests/golden/make_full_scale.py [name ...]   ->  tests/golden/full_scale.json
    python tests/golden/make_full_scale.py --orders       ->  full_scale.json["logit1b"]["orders"]

`--orders` records, beside the compensated trajectory the engine reproduces, the logit1b fit with
the reference's own summation order for the deviance (plain per-partition running sums, the
partitions added in order: GLM.scala:168, 404-407) and, to separate the two effects, the same
8-partition fitMultipleBinomial with compensated sums.
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po  # noqa: E402  (the checker)

# name -> (kind, row0, n, p, seed, family, link): bench.py WORKLOADS at their full sizes
CASES = {
    "logit1b": (0, 0, 1_000_000_000, 32, 6, "binomial", "logit"),      # north-star strong-scaling fit
    "logit256": (0, 0, 100_000_000, 256, 2, "binomial", "logit"),      # BASELINE configs[1] (headline)
    "poisson64": (2, 0, 125_000_000, 64, 3, "poisson", "log"),         # configs[2] per-GPU shard
    "logit512r": (0, 0, 60_000_000, 512, 5, "binomial", "logit"),      # configs[4] p, resident: the wide path
    "gamma2048": (3, 0, 12_500_000, 2048, 4, "gamma", "inverse"),     # configs[3] per-GPU shard, wide + GPU solve
    "logit512p": (0, 0, 250_000_000, 512, 5, "binomial", "logit"),     # configs[4] per-GPU shard, procedural X
}
PROCEDURAL = {"logit512p"}


def orders(out):
    kind, row0, n, p, seed, fam, link = CASES["logit1b"]
    res = {}
    for label, plain in (("reference_order_npart8", True), ("compensated_npart8", False)):
        t0 = time.time()
        f = po.fit_glm_synth(kind, row0, n, p, seed, fam, link, nthreads=os.cpu_count() or 8, npart=8,
                             plain_sums=plain, verbose=True)
        res[label] = {"npart": 8, "init": "multiple", "plain_sums": plain, "iter": f.iter, "coefs": f.coefs.tolist(),
                      "stderr": f.stderr.tolist(), "deviance": f.deviance, "dev_trace": f.dev_trace.tolist(),
                      "oracle_seconds": round(time.time() - t0, 1)}
        print(f"logit1b {label}: {f.iter} iterations, deltas {[b - a for a, b in zip(f.dev_trace, f.dev_trace[1:])]}",
              flush=True)
    out["logit1b"]["orders"] = res


def main(names):
    path = os.path.join(HERE, "full_scale.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    if names == ["--orders"]:
        orders(out)
        with open(path, "w") as fh:
            json.dump(out, fh, indent=1)
        return
    for name in names or list(CASES):
        kind, row0, n, p, seed, fam, link = CASES[name]
        t0 = time.time()
        f = po.fit_glm_synth(kind, row0, n, p, seed, fam, link, nthreads=os.cpu_count() or 8, verbose=True)
        dt = time.time() - t0
        out[name] = {"kind": kind, "row0": row0, "n": n, "p": p, "seed": seed, "family": fam, "link": link,
                     "tol": 1e-6, "init": "single", "iter": f.iter, "coefs": f.coefs.tolist(),
                     "stderr": f.stderr.tolist(), "deviance": f.deviance, "null_deviance": f.null_deviance,
                     "pearson": f.pearson, "loglik": f.loglik, "dev_trace": f.dev_trace.tolist(),
                     "oracle_seconds": round(dt, 1), "procedural": name in PROCEDURAL}
        print(f"{name}: {f.iter} iterations, deviance {f.deviance!r}, {dt:.0f} s", flush=True)
        with open(path, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
