"""Run-to-run determinism of every pass kernel family: the same IRLS pass at the same beta, repeated
in one process, must give bitwise the same X'WX, X'Wz and scalars (the partials are reduced in a
fixed order, so any difference is a race -- e.g. a row stage reading an LDS-DMA image that has not
landed).  Sizes are large enough that every wave streams many blocks, and the families with an eta
store (Poisson, Gaussian; the IRLS passes that do not carry the final statistics) are included: their
extra vector-memory store shifts the vmcnt accounting of the narrow kernels' DMA pipeline.

Round 5 found exactly that in the p > 32 block-pair loop of irls_narrow_kernel (a wait that counted
the eta store as younger than the next block's DMA): ~1e-6 relative run-to-run differences in the
Poisson + offset + prior and Gaussian passes at p = 48 / 64 (narrow.hip pair_blocks)."""
import numpy as np
import pytest

from sparkglm_amd import Engine

pytestmark = pytest.mark.gpu

CASES = [
    # (rows, p, synth kind, family, link): the kernel the engine picks for that shape
    (20_000_000, 64, 2, "poisson", "log"),       # irls_narrow_kernel<4>, pairs of 16-row blocks, eta store
    (20_000_000, 48, 2, "poisson", "log"),       # irls_narrow_kernel<3>
    (20_000_000, 64, 1, "gaussian", "identity"),  # irls_narrow_kernel<4>, w = 1
    (20_000_000, 40, 0, "binomial", "logit"),    # irls_narrow_kernel<3>, statistics in the pass, no eta store
    (30_000_000, 32, 2, "poisson", "log"),       # irls_narrow_kernel<2>, pairs of 32-row blocks, eta store
    (30_000_000, 20, 1, "gaussian", "identity"),  # irls_narrow_kernel<2>
    (30_000_000, 32, 0, "binomial", "probit"),   # irls_narrow_kernel<2>, reference-order row path
    (4_000_000, 96, 2, "poisson", "log"),        # K1<6>
    (3_000_000, 256, 0, "binomial", "logit"),    # K1r<16>
    (2_000_000, 160, 3, "gamma", "inverse"),     # K1r<10>
    (500_000, 512, 0, "binomial", "logit"),      # wide path
]


@pytest.mark.parametrize("n,p,kind,family,link", CASES)
def test_pass_is_bitwise_repeatable(n, p, kind, family, link):
    with Engine(0) as e:
        e.synth(kind, 0, n, p, 11)
        b = np.linspace(-0.02, 0.02, p)
        if kind == 3:
            b[0] = 1.0  # the gamma design's positive linear predictor
        runs = [e.irls_pass(b, family=family, link=link) for _ in range(4)]
        kern = e.stats()["pass_kernel_name"]
    for r in runs[1:]:
        for part, a0, a in zip(("X'WX", "X'Wz", "scalars"), runs[0], r):
            d = np.abs(np.asarray(a) - np.asarray(a0))
            assert np.array_equal(np.asarray(a), np.asarray(a0)), (
                f"{kern}: {part} differs run to run in {np.count_nonzero(d)} entries, max |diff| {d.max():.3e}")
