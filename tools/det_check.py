"""Run-to-run determinism of one IRLS pass (development tool).
usage: python tools/det_check.py n:p:kind:family:link [...]
For each case: the same pass at a fixed beta, three times in one process, then the entries that differ
between runs (X'WX, X'Wz, scalars) with their absolute size against the largest entry of their part."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkglm_amd import Engine  # noqa: E402


def main():
    for spec in sys.argv[1:]:
        n, p, k, fam, lnk = spec.split(":")
        n, p, k = int(n), int(p), int(k)
        with Engine(0) as e:
            e.synth(k, 0, n, p, 2)
            b = np.linspace(-0.02, 0.02, p)
            outs = [e.irls_pass(b, family=fam, link=lnk) for _ in range(3)]
            st = e.stats()
        kern = st.get("pass_kernel_name")
        for name, i in (("gram", 0), ("xz", 1), ("scalars", 2)):
            a = [np.ravel(o[i]) for o in outs]
            scale = max(float(np.max(np.abs(a[0]))), 1e-300)
            for r in (1, 2):
                d = np.abs(a[r] - a[0])
                nd = int(np.count_nonzero(d))
                if nd:
                    j = int(np.argmax(d))
                    print(f"{spec} {kern} {name}: run {r} differs in {nd}/{d.size} entries, max |diff| {d[j]:.3e} "
                          f"at {j} (value {a[0][j]:.6e}; part max {scale:.3e}, rel to max {d[j] / scale:.2e})",
                          flush=True)
                else:
                    print(f"{spec} {kern} {name}: run {r} bitwise", flush=True)


if __name__ == "__main__":
    main()
