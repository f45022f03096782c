"""The device generator's integer construction of the design's affine maps (procx.hpp affine_u) is
bit for bit synth.py's fp64 expressions (2u - 1) and (0.5 + u), u = (h >> 11) 2^-53.  This restates
affine_u in numpy uint64 ops and checks it on random hashes and on the edge patterns (r = 0, r all
ones, both values of bit 63, the rounding ties of 0.5 + u); the GPU tests check the device code
itself (procedural fits bitwise the host-generated resident ones, tests/test_gpu_wide.py)."""
import numpy as np

from sparkglm_amd import synth

MANT = np.uint64(0xFFFFFFFFFFFFF)


def _affine_bits(h, pos):
    h = np.asarray(h, dtype=np.uint64)
    e = np.uint64(0x3FE if pos else 0x3FF)
    d = ((e << np.uint64(52)) | ((h >> np.uint64(11)) & MANT)).view(np.float64)
    b = (h >> np.uint64(63)) != 0
    if pos:
        c = np.where(b, np.uint64(0x3FE0000000000000), np.uint64(0))
    else:
        c = np.where(b, np.uint64(0xBFF0000000000000), np.uint64(0xC000000000000000))
    return d + c.astype(np.uint64).view(np.float64)


def _formula(h, pos):
    u = (np.asarray(h, dtype=np.uint64) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
    return (0.5 + u) if pos else (2.0 * u - 1.0)


def _hashes():
    rng = np.random.default_rng(7)
    h = rng.integers(0, 2 ** 63, size=2_000_000, dtype=np.uint64) * np.uint64(2) + \
        rng.integers(0, 2, size=2_000_000, dtype=np.uint64)
    low = np.arange(4096, dtype=np.uint64)  # bits below 11 are dropped; r = 0 with b = 0
    edges = []
    for b in (0, 1):
        for r in (0, 1, 2, 3, (1 << 52) - 1, (1 << 52) - 2, 1 << 51, (1 << 51) + 1):
            edges.append(((b << 63) | (r << 11)) & ((1 << 64) - 1))
    return np.concatenate([h, low, np.array(edges, dtype=np.uint64), synth.splitmix64(np.arange(100_000))])


def test_affine_maps_are_bitwise_the_fp64_formula():
    h = _hashes()
    for pos in (False, True):
        got, want = _affine_bits(h, pos), _formula(h, pos)
        assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), pos
