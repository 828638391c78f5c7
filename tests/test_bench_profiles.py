"""The bench line's roofline recomputes from the committed evidence under profiles/r03/ (VERDICT r2
item 2): the rocprofv3 kernel-trace summary gives the dominant step kernel's average launch
duration, the FETCH_SIZE / WRITE_SIZE summary its HBM bytes per launch, and the committed bench
line's `frac` equals SURVEY §8d's FLOPs per launch over that duration."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
bench = pytest.importorskip("bench")


def _line():
    with open(os.path.join(ROOT, "profiles", "r03", "bench_plain.json")) as fh:
        return json.loads(fh.read().strip().splitlines()[-1])


def test_step_flops_config2():
    """§8d per-launch FLOPs of config 2's step at B = 200 (d = 8, R = 1024, P = 2048, g = 8, 8, 1)."""
    fwd, bwd = bench.step_flops(200, [8, 8, 8], [1024] * 3, [2048] * 3, [8, 8, 1])
    assert sum(fwd) + sum(bwd) == pytest.approx(51.6e6, rel=2e-3)
    assert sum(bwd) / 3 == pytest.approx(9_284_266, abs=1)


def test_roofline_recomputes_from_profiles():
    line = _line()
    roof = line["roofline"]
    us = bench.rocprof_avg_us(roof["kernel"])
    assert us is not None and us > 0
    frac = roof["flops_per_launch"] / (us * 1e-6) / (bench.FP32_MFMA_PEAK)
    # the committed line was taken with the trace present: its frac is this recomputation
    # (within 5 %: the trace summary may have been refreshed after the line)
    assert roof["frac"] == pytest.approx(frac, rel=0.05)
    traffic = bench.pmc_traffic(roof["kernel"])
    assert traffic is not None and traffic > 0
    assert roof["traffic"] == traffic


def test_secondary_ceilings_present():
    line = _line()
    lf = line["roofline"]["launch_floor"]
    assert lf["launches_per_step"] == 7 and lf["boundary_us"] > 0
    tc = line["roofline_predictive"]["transcendental_ceiling"]
    assert tc["sin_cos_per_sample"] == 100_000 * 2 * 3 * 1024
    assert 0 < tc["frac_of_sample_time"] < 1
    assert set(line["b_sweep"]) == {"200", "1024", "8192", "65536"}
