"""The engine's kernel choice (sglm_pass_kernel_for: the rule ensure_workspace / launch_pass /
launch_narrow apply, and the label of bench.py's roofline line) -- on the CPU, no device touched:
narrow for p <= 64; the fused pass for 65 <= p <= 256: P16 = ceil(p / 16) column blocks, split-role K1r
from P16 = 10 and at every odd P16 >= 9; K1 below, at odd 5 and 7 too (its tiles are runs of the tile
sequence); an odd count >= 9 that may not run K1r rounds up to K1's next even one; SGLM_FUSED_SPLIT =
5 / 7 puts K1r on the odd counts below) unless SGLM_FUSED_SPLIT moves or disables the threshold, and K1 again when
the shard is too tall for K1r's 32-bit DMA lane offsets (ld * 24 + 4096 >= 2^32, ~179M rows); the
wide path above p = 256, for procedural shards and under SGLM_FORCE_WIDE."""
import pytest

from sparkglm_amd import _lib as L


@pytest.mark.parametrize("n,p,fs,proc,force,kind,name", [
    (1_000_000, 20, 1, False, False, "narrow", "irls_narrow_kernel<2,binomial,logit>"),
    (1_000_000_000, 32, 1, False, False, "narrow", "irls_narrow_kernel<2,binomial,logit>"),
    (125_000_000, 64, 1, False, False, "narrow", "irls_narrow_kernel<4,binomial,logit>"),
    (125_000_000, 48, 1, False, False, "narrow", "irls_narrow_kernel<3,binomial,logit>"),
    (125_000_000, 33, 1, False, False, "narrow", "irls_narrow_kernel<3,binomial,logit>"),
    (600_000_000, 64, 1, False, False, "narrow", "irls_narrow_kernel<4,binomial,logit>"),
    (10_000_000, 65, 1, False, False, "fused", "irls_pass_kernel<5,binomial,logit>"),
    (10_000_000, 80, 1, False, False, "fused", "irls_pass_kernel<5,binomial,logit>"),
    (10_000_000, 80, 5, False, False, "fused-split", "irls_pass_r_kernel<5,binomial,logit>"),
    (10_000_000, 81, 1, False, False, "fused", "irls_pass_kernel<6,binomial,logit>"),
    (10_000_000, 80, 0, False, False, "fused", "irls_pass_kernel<5,binomial,logit>"),  # K1 runs odd 5 / 7
    (10_000_000, 80, 6, False, False, "fused", "irls_pass_kernel<5,binomial,logit>"),  # K1r from 6: K1 at odd 5
    (10_000_000, 96, 6, False, False, "fused-split", "irls_pass_r_kernel<6,binomial,logit>"),
    (10_000_000, 112, 1, False, False, "fused", "irls_pass_kernel<7,binomial,logit>"),
    (10_000_000, 112, 7, False, False, "fused-split", "irls_pass_r_kernel<7,binomial,logit>"),
    (10_000_000, 144, 1, False, False, "fused-split", "irls_pass_r_kernel<9,binomial,logit>"),
    (10_000_000, 128, 1, False, False, "fused", "irls_pass_kernel<8,binomial,logit>"),
    (10_000_000, 129, 1, False, False, "fused-split", "irls_pass_r_kernel<9,binomial,logit>"),
    (10_000_000, 240, 1, False, False, "fused-split", "irls_pass_r_kernel<15,binomial,logit>"),
    (180_000_000, 140, 1, False, False, "fused", "irls_pass_kernel<10,binomial,logit>"),  # odd, too tall for K1r
    (10_000_000, 160, 1, False, False, "fused-split", "irls_pass_r_kernel<10,binomial,logit>"),
    (100_000_000, 256, 1, False, False, "fused-split", "irls_pass_r_kernel<16,binomial,logit>"),
    (100_000_000, 256, 0, False, False, "fused", "irls_pass_kernel<16,binomial,logit>"),
    (10_000_000, 96, 6, False, False, "fused-split", "irls_pass_r_kernel<6,binomial,logit>"),
    (10_000_000, 160, 12, False, False, "fused", "irls_pass_kernel<10,binomial,logit>"),
    (178_000_000, 160, 1, False, False, "fused-split", "irls_pass_r_kernel<10,binomial,logit>"),
    (180_000_000, 160, 1, False, False, "fused", "irls_pass_kernel<10,binomial,logit>"),  # K1r's row limit
    (200_000_000, 256, 1, False, False, "fused", "irls_pass_kernel<16,binomial,logit>"),
    (60_000_000, 512, 1, False, False, "wide", "wide_gram_kernel<resident>"),
    (250_000_000, 512, 1, True, False, "wide-procedural", "wide_gram_kernel<procedural>"),
    (6000, 40, 1, True, False, "wide-procedural", "wide_gram_kernel<procedural>"),
    (6000, 40, 1, False, True, "wide", "wide_gram_kernel<resident>"),
])
def test_kernel_choice(n, p, fs, proc, force, kind, name):
    assert L.pass_kernel_for(n, p, fused_split=fs, procedural=proc, force_wide=force) == (kind, name)


@pytest.mark.parametrize("n,p", [(125_000_000, 64), (125_000_000, 33), (1_000_000_000, 32), (536_870_912, 64),
                                 (1_000_000, 16)])
def test_every_narrow_shard_runs_the_narrow_kernel(n, p):
    # p <= 64 at any shard height: irls_narrow_kernel (the split-role narrow pass, measured 30-44 %
    # slower on MI355X, was removed in round 6)
    P16 = (p + 15) // 16
    assert L.pass_kernel_for(n, p) == ("narrow", f"irls_narrow_kernel<{P16},binomial,logit>")


def test_kernel_name_carries_the_family():
    assert L.pass_kernel_for(125_000_000, 64, "poisson", "log")[1] == "irls_narrow_kernel<4,poisson,log>"
    assert L.pass_kernel_for(1_000_000, 200, "gamma", "inverse")[1] == "irls_pass_r_kernel<13,gamma,inverse>"


def test_bad_arguments_are_refused():
    with pytest.raises(L.IllegalArgumentException):
        L.pass_kernel_for(0, 10)
    with pytest.raises(L.IllegalArgumentException):
        L.pass_kernel_for(10, 10, "poisson", "logit")
