"""The bench line's roofline and its committed evidence (bench.PROFILES = profiles/r06/): the line's
`frac` is SURVEY §8d's FLOPs per launch over the dominant step kernel's dispatch-weighted mean
duration in the committed rocprofv3 kernel-trace summary of the same command (recomputed here); the
live in-kernel span the command measured must sit within the trace's per-dispatch overhead of it;
the FETCH_SIZE / WRITE_SIZE summary gives its bytes per launch."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
bench = pytest.importorskip("bench")


def _line():
    path = os.path.join(bench.PROFILES, "bench_plain.json")
    if not os.path.exists(path):
        pytest.skip(f"{os.path.relpath(path, ROOT)} not committed yet")
    with open(path) as fh:
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
    """The traced run is slower than the plain one (tracing adds a completion signal per dispatch):
    its own step time (`trace_step_us`, from the committed bench_under_rocprof.json) is within 1.5x
    of the plain run's; the dominant kernel's traced duration rescaled by plain / traced step time
    agrees with the live in-kernel span (hipEvent pair minus an empty pair, same command) to 25 %,
    and the live span lies between the traced duration minus the tracer's per-dispatch overhead
    (the traced duration of the one-thread k_advance) and the traced duration."""
    roof = _line()["roofline"]
    us = bench.rocprof_avg_us(roof["kernel"])
    ovh = bench.rocprof_avg_us("k_advance")
    assert ovh is not None and 0 < ovh < us
    assert roof["trace_dispatch_overhead_us"] == pytest.approx(ovh, rel=1e-3)
    with open(os.path.join(bench.PROFILES, "bench_under_rocprof.json")) as fh:
        traced = json.loads(fh.read().strip().splitlines()[-1])["roofline"]
    assert roof["trace_step_us"] == pytest.approx(traced["step_us_events"], rel=1e-6)
    assert roof["step_us_events"] <= roof["trace_step_us"] <= 1.5 * roof["step_us_events"]
    scaled = us * roof["step_us_events"] / roof["trace_step_us"]
    assert roof["rocprof_scaled_us"] == pytest.approx(scaled, rel=1e-3)
    assert abs(roof["live_in_kernel_us"] - scaled) <= 0.15 * scaled
    assert us - ovh <= roof["live_in_kernel_us"] <= us
    traffic = bench.pmc_traffic(roof["kernel"])
    assert traffic is not None and traffic > 0
    assert roof["traffic"] == traffic


def _fracs(obj, path=""):
    if isinstance(obj, dict):
        for k, v in obj.items():
            if "frac" in k and isinstance(v, (int, float)):
                yield f"{path}.{k}", v
            yield from _fracs(v, f"{path}.{k}")
    elif isinstance(obj, list):
        for i, v in enumerate(obj):
            yield from _fracs(v, f"{path}[{i}]")


def test_no_fraction_above_one():
    """Every MFMA / roofline fraction on the line (step, predictive, configs 3-5, B-sweep) is in
    (0, 1]: each is computed from the FLOPs its timed region executes."""
    fr = dict(_fracs(_line()))
    assert any("predictive_mfma_frac" in k for k in fr) and any("step_mfma_frac" in k for k in fr)
    bad = {k: v for k, v in fr.items() if not 0 < v <= 1}
    assert not bad, bad


def test_secondary_ceilings_present():
    line = _line()
    lf = line["roofline"]["launch_floor"]
    assert lf["launches_per_step"] in (6, 7) and lf["boundary_us"] > 0
    tc = line["roofline_predictive"]["transcendental_ceiling"]
    # layer 0's cos / sin once per pair of samples (the pair kernel), layers 1-2 per sample
    assert tc["sin_cos_per_sample"] == 100_000 * (1024 + 2 * 2 * 1024)
    assert 0 < tc["frac_of_sample_time"] < 1
    assert set(line["b_sweep"]) == {"200", "1024", "8192", "65536"}
