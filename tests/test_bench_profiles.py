"""The bench line's roofline and its committed evidence (bench.PROFILES = profiles/r04/): the line's
`frac` is SURVEY §8d's FLOPs per launch over the live hipEvent duration of the dominant step kernel;
the committed rocprofv3 kernel-trace summary of the same command gives that kernel's traced average
duration (`rocprof_avg_launch_us`, recomputed here), which must agree with the live figure up to the
dispatch overhead a trace adds; the FETCH_SIZE / WRITE_SIZE summary gives its bytes per launch."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
bench = pytest.importorskip("bench")


def _line():
    with open(os.path.join(bench.PROFILES, "bench_plain.json")) as fh:
        return json.loads(fh.read().strip().splitlines()[-1])


def test_step_flops_config2():
    """§8d per-launch FLOPs of config 2's step at B = 200 (d = 8, R = 1024, P = 2048, g = 8, 8, 1)."""
    fwd, bwd = bench.step_flops(200, [8, 8, 8], [1024] * 3, [2048] * 3, [8, 8, 1])
    assert sum(fwd) + sum(bwd) == pytest.approx(51.6e6, rel=2e-3)
    assert sum(bwd) / 3 == pytest.approx(9_284_266, abs=1)


def test_roofline_frac_recomputes_from_committed_trace():
    """`frac` = §8d FLOPs per launch / the committed trace's dispatch-weighted mean duration of
    the dominant kernel / the fp32 MFMA peak, to 1e-3."""
    roof = _line()["roofline"]
    us = bench.rocprof_avg_us(roof["kernel"])
    assert us is not None and us > 0
    frac = roof["flops_per_launch"] / (us * 1e-6) / bench.FP32_MFMA_PEAK
    assert roof["frac"] == pytest.approx(frac, rel=1e-3)
    assert roof["avg_launch_us"] == pytest.approx(us, rel=1e-3)
    assert roof["achieved"] == pytest.approx(frac * bench.FP32_MFMA_PEAK / 1e12, rel=1e-3)


def test_committed_trace_agrees_with_live():
    roof = _line()["roofline"]
    us = bench.rocprof_avg_us(roof["kernel"])
    # the live in-kernel span (hipEvent pair minus an empty pair) measured by the same command
    # agrees with the traced duration within 15 %
    assert roof["live_in_kernel_us"] == pytest.approx(us, rel=0.15)
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
