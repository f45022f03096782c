"""configs[3]'s conditioning floor (oracle/lu_floor.py): on the SAME X'WX -- the oracle's own, of
a fit's last solve -- LAPACK's dgetrf + dgetri (Breeze inv as netlib-java binds a native LAPACK),
the Cholesky route and a re-summed X'WX land ~cond * eps apart.  The committed p = 2048 run
(tests/golden/lu_floor_p2048.json, 100 s on 8 cores) shows that spread above 1e-9 on the smallest
coefficients: the reference itself defines them no better.  Here the script is
exercised at p = 256 (CPU only, seconds) and the committed numbers are checked for what DESIGN.md
quotes."""
import json
import os

import lu_floor
from conftest import GOLDEN


def test_lu_floor_machinery_small():
    out = lu_floor.run(n=2500, p=256)
    # stdErr is the oracle's own diag bitwise; inv * b summed by BLAS instead of in the oracle's order
    # already moves the smallest coefficient by ~4e-10 at cond 1.5e4 (cancellation in the product)
    assert out["oracle_reproduces_fit"]["stderr"] == 0.0 and out["oracle_reproduces_fit"]["coefs"] < 1e-9
    for k in ("lapack", "lapack_solve", "chol", "gram_blas"):
        assert out[k]["coefs_nrel"] < 1e-11 and out[k]["stderr_rel"] < 1e-11, (k, out[k])


def test_committed_p2048_floor():
    out = json.load(open(os.path.join(GOLDEN, "lu_floor_p2048.json")))
    assert out["p"] == 2048 and out["cond"] > 1e5
    # the reference's own algorithm, two implementations, the same matrix: > 1e-9 apart elementwise,
    # < 1e-11 norm-wise
    assert out["lapack"]["coefs_rel"] > 1e-9 and out["gram_blas"]["coefs_rel"] > 1e-9
    for k in ("lapack", "lapack_solve", "chol", "gram_blas"):
        assert out[k]["coefs_nrel"] < 1e-11 and out[k]["stderr_rel"] < 1e-11
