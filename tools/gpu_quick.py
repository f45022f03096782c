"""Quick GPU sanity run (development tool): engine vs oracle on small cases + timing."""
import sys, time, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import pyoracle as po
from sparkglm_amd import Engine
from sparkglm_amd import synth

def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))

e = Engine(0)
# 1. synth bit-identity
for kind in (0, 1, 2):
    e.synth(kind, 12345, 1000, 20, 7)
    X, y, m, off, pr = e.get_data()
    Xh, yh, oh, ph = synth.generate(kind, 12345, 1000, 20, 7)
    ok = np.array_equal(X, Xh) and np.array_equal(y, yh)
    if kind == 2:
        ok = ok and np.array_equal(off, oh) and np.array_equal(pr, ph)
    print("synth", kind, "bit-identical:", ok, flush=True)

# 2. Gram vs numpy for several p
rng = np.random.default_rng(0)
for p in (3, 16, 20, 33, 64, 100, 128, 200, 256):
    n = 5000 + p
    X = rng.uniform(-1, 1, (n, p)); X[:, 0] = 1
    y = (rng.uniform(size=n) < 0.4).astype(float)
    e.set_data(X, y)
    beta = rng.normal(size=p) * 0.1
    G, xz, s = e.irls_pass(beta)
    eta = X @ beta; mu = 1 / (1 + np.exp(-eta)); g = 1 / (mu * (1 - mu)); w = 1 / (mu * (1 - mu) * g * g)
    z = eta + (y - mu) * g
    Gr = (X * w[:, None]).T @ X; xzr = X.T @ (w * z)
    print(f"p={p:4d} gram rel {rel(G, Gr):.2e} xtwz rel {rel(xz, xzr):.2e} stats {e.stats()['kernel_variant']}", flush=True)

# 3. full logit fit vs oracle
n, p = 20000, 12
X = rng.uniform(-1, 1, (n, p)); X[:, 0] = 1
bt = rng.normal(size=p)
y = (rng.uniform(size=n) < 1 / (1 + np.exp(-X @ bt))).astype(float)
for link in ("logit", "probit", "cloglog"):
    e.set_data(X, y)
    f = e.fit_glm("binomial", link)
    o = po.fit_glm(X, y, "binomial", link)
    print(link, "iter", f.iter, o.iter, "coef", rel(f.coefs, o.coefs), "se", rel(f.stderr, o.stderr),
          "dev", rel(f.deviance, o.deviance), "ll", rel(f.loglik, o.loglik), "pear", rel(f.pearson, o.pearson), flush=True)

# 4. LM iris-like
Xl = np.column_stack([np.ones(1000), rng.normal(size=(1000, 5))]); yl = Xl @ rng.normal(size=6) + rng.normal(size=1000)
e.set_data(Xl, yl); fl = e.fit_lm(); ol = po.fit_lm(Xl, yl)
print("lm coef", rel(fl.coefs, ol["coefs"]), "se", rel(fl.stderr, ol["stderr"]), "r2", rel(fl.r2, ol["r2"]), flush=True)

# 5. timing at 10M x 256
n, p = int(os.environ.get("QN", "10000000")), 256
t0 = time.time(); e.synth(0, 0, n, p, 2); print("synth s", time.time() - t0, flush=True)
t0 = time.time(); f = e.fit_glm("binomial", "logit"); print("fit s", time.time() - t0, "iter", f.iter, f.dev_trace, flush=True)
st = e.stats(); print(st, flush=True)
per = st["pass_kernel_ms"] / st["passes"]
flops = n * (p * (p + 1) + 2 * p)
print(f"pass ms {per:.3f}  TFLOP/s {flops / per / 1e9:.2f}  GB/s {n * 8 * (p + 1) / per / 1e6:.1f}", flush=True)
