"""Host-side logic of bench.py (no GPU): the roofline it reports is computed
from the committed counter passes of the timed launch shape, stays <= 1, and
the CPU baseline sizes itself to the cores this process may use."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


@pytest.mark.parametrize("steps", [20, 200])
def test_committed_counter_passes_give_executed_roofline(steps):
    e = bench.pmc_entry("C3-dof53-b65536", steps)
    assert e.get("epochs_per_launch") == steps, "no counter pass of the %d-epoch launch committed" % steps
    pw = e["per_wave_epoch"]
    # the counters come from the timed launch of 65,536 instances (normalised per
    # instance-epoch; the tail spreading adds chunk waves beyond one per instance)
    assert e["instances"] == 65536
    assert 65536 <= e["waves"] <= 65536 + 8 * 7 * 8 * 384
    assert 0 < pw["valu_fma_f64"] < pw["valu"]
    # a plausible kernel time for that shape (0.43-0.5 ms per epoch): frac stays in (0, 1)
    for ms in (0.43 * steps, 0.5 * steps):
        cr = bench.counter_roofline(e, 65536, steps, ms)
        frac = cr["achieved_tflops"] / bench.PEAK_FP64_TFLOPS
        assert 0.1 < frac < 1.0
    assert 0 < e["valu_busy"]["model_frac"] <= e["valu_busy"]["frac"] <= 1.0
    # traffic: at least the packed Sigma + mu round trip of every instance
    assert e["bytes_per_launch"] >= 65536 * 2 * (1431 + 54) * 8 * 0.95


def test_pmc_entry_falls_back_without_exact_shape():
    assert bench.pmc_entry("C3-dof53-b65536", 12345).get("epochs_per_launch") != 12345
    assert bench.pmc_entry("no-such-workload", 20) == {}


def test_available_cores_and_torchrun_detection(monkeypatch):
    n = bench.available_cores()
    assert 1 <= n <= (os.cpu_count() or 1)
    for k in ("TORCHELASTIC_RUN_ID", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    assert not bench.launched_by_torchrun()
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "x")
    assert bench.launched_by_torchrun()


def test_flop_models():
    assert bench.F_STEP == 1_554_084  # SURVEY 8(d), frozen
    assert 40_000 < bench.F_STEP_PSP < 70_000  # the PSP engine's own model


def test_bench_line_fields_documented():
    """The keys the driver and the judge read are the ones DESIGN.md section 6 documents."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    for key in ('"roofline"', '"cpu_baseline"', '"achieved"', '"peak"', '"frac"', '"traffic"',
                '"effective_tflops"', '"counters"', '"timing"'):
        assert key in src
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    assert "C3-dof53-b65536-e20" in d
