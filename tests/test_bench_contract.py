"""bench.py's contract pieces that need no GPU: every workload maps to a BASELINE.json config
with the family / shape it names, the traffic lookup, and the roofline bound choice."""
import importlib.util
import json
import os

from conftest import ROOT

spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)


def test_workloads_follow_baseline_configs():
    cfgs = json.load(open(os.path.join(ROOT, "BASELINE.json")))["configs"]
    assert bench.WORKLOADS["logit256"]["cfg"] == 1  # the default = the headline config
    for name, wl in bench.WORKLOADS.items():
        text = cfgs[wl["cfg"]].lower()
        fam = wl["family"].lower()
        assert fam in text or (fam == "binomial" and "logit" in text), name
        if wl.get("strong_rows") is None:
            assert str(wl["p"]) in text.replace("×", "x"), name
    assert bench.WORKLOADS["logit512"]["procedural"] is True  # 2B x 512 cannot be resident
    assert bench.WORKLOADS["logit1b"]["strong_rows"] == 1_000_000_000


def test_roofline_bound_follows_arithmetic_intensity():
    # flops p(p+1)+2p, bytes 8p + 8k per row; ridge = 78.6 TF / 8 TB/s
    def bound(p, nvec):
        return "hbm" if (p * (p + 1) + 2 * p) / (8 * p + 8 * nvec) < bench.RIDGE else "mfma"
    assert bound(64, 3) == "hbm" and bound(32, 1) == "hbm"
    assert bound(256, 1) == "mfma" and bound(512, 1) == "mfma" and bound(2048, 1) == "mfma"


def test_pmc_traffic_lookup():
    t = bench.pmc_traffic(256, 1000, "binomial")
    assert t is not None and 2000 * 1000 < t < 2200 * 1000
    assert bench.pmc_traffic(512, 10, "binomial", procedural=True) < bench.pmc_traffic(512, 10, "binomial")
    assert bench.pmc_traffic(333, 10, "binomial") is None


def test_every_baseline_config_has_a_workload():
    cfgs = json.load(open(os.path.join(ROOT, "BASELINE.json")))["configs"]
    assert {wl["cfg"] for wl in bench.WORKLOADS.values()} == set(range(len(cfgs)))
    assert bench.WORKLOADS["lm20"]["cfg"] == 0 and bench.WORKLOADS["lm20"].get("lm")


def test_strong_scaling_point_and_p32_traffic():
    # the default run appends the north-star 1B x 32 strong-scaling point (bench.strong_1b),
    # whose per-row PMC traffic the logit1b roofline uses
    assert callable(bench.strong_1b) and callable(bench.attach_comm)
    t = bench.pmc_traffic(32, 1000, "binomial")
    assert t is not None and 264 * 1000 <= t < 280 * 1000
