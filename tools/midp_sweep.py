"""Mid-width fused-pass sweep: for each p, a ~24 GB synthetic logit design, one
warm-up pass and K timed passes; prints the engine's kernel label, ms per pass, algorithmic TF/s
(SYRK convention p(p+1) + 2p flops per row) against the 78.6 TF/s fp64 MFMA peak, and the HBM rate of
the pass bytes (8p + 8 per row) against 8 TB/s -- p = 80 sits at the ridge, so both are printed.
    python tools/midp_sweep.py [p ...]      (run under rocprofv3 --kernel-trace --stats for the CSV)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sparkglm_amd import Engine  # noqa: E402

PEAK_TF, PEAK_GBS = 78.6, 8000.0


def main():
    ps = [int(a) for a in sys.argv[1:]] or [80, 96, 112, 128, 144, 160, 192, 224, 240, 256]
    k = int(os.environ.get("SWEEP_PASSES", "5"))
    for p in ps:
        n = int(24e9 / (8 * p)) // 32 * 32
        with Engine(0) as e:
            e.synth(0, 0, n, p, 2)
            b = np.full(p, 0.01)
            e.irls_pass(b)
            e.reset_stats()
            for _ in range(k):
                e.irls_pass(b)
            st = e.stats()
        ms = st["pass_kernel_ms"] / st["passes"]
        tf = n * (p * (p + 1) + 2 * p) / (ms * 1e-3) / 1e12
        gbs = n * (8 * p + 8) / (ms * 1e-3) / 1e9
        print(f"p={p:4d} n={n:11d} {st['pass_kernel_name']:40s} {ms:8.3f} ms  {tf:5.1f} TF/s = {100 * tf / PEAK_TF:5.1f} % MFMA"
              f"  {gbs:6.0f} GB/s = {100 * gbs / PEAK_GBS:5.1f} % HBM", flush=True)


if __name__ == "__main__":
    main()
