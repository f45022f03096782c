"""Host wall time of LM.fit on the configs[0] design (1M x 20, resident), fit by fit, and a rough
split of where it goes: python tools/lm_timeline.py [fits].  Run under rocprofv3 --kernel-trace
--memory-copy-trace to line the kernels and copies up against the host calls."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sparkglm_amd import Engine  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    with Engine(0) as e:
        e.synth(1, 0, 1_000_000, 20, 1)
        for _ in range(20):
            e.fit_lm()
        e.reset_stats()
        t = []
        for _ in range(k):
            t0 = time.perf_counter()
            e.fit_lm()
            t.append(time.perf_counter() - t0)
        st = e.stats()
        # the same fit's GPU stages, one by one
        g = []
        for _ in range(k):
            t0 = time.perf_counter()
            e.irls_pass(None, mu0=0.0, family="gaussian", link="identity")
            g.append(time.perf_counter() - t0)
    t, g = np.array(t) * 1e3, np.array(g) * 1e3
    print(f"fit_lm: median {np.median(t):.4f} ms, min {t.min():.4f} ms over {k} fits; "
          f"Gram pass kernel {st['pass_kernel_ms'] / st['passes']:.4f} ms, reduce {st['reduce_kernel_ms'] / st['passes']:.4f} ms; "
          f"an init-mode pass round trip (sglm_irls_pass) median {np.median(g):.4f} ms")


if __name__ == "__main__":
    main()
