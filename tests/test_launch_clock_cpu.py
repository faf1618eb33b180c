"""Arithmetic of the in-run launch clock (device.clock_summary over the
rt_clock_stamps words); the stamps themselves are checked on the GPU in
tests/test_launch_clock_gpu.py."""
import pytest


def test_clock_summary_arithmetic():
    from reticulum_amd.device import clock_summary
    # 20 launches x 256 workgroups, each 1.95 M cycles over 0.88 ms (88 000 ticks)
    wgs, launches = 20 * 256, 20
    words = [wgs * 1_950_000, wgs * 88_000, wgs, launches, 0, 0, 0, 0]
    s = clock_summary(words)
    assert set(s) == {"encrypt"}
    e = s["encrypt"]
    assert e["clock_ghz"] == pytest.approx(1.95e6 / 0.88e-3 / 1e9)
    assert e["cycles_per_launch"] == pytest.approx(1.95e6)
    assert e["wg_span_ms"] == pytest.approx(0.88)
    assert e["launches"] == 20 and e["workgroups_per_launch"] == 256


def test_clock_summary_both_kernels_and_empty():
    from reticulum_amd.device import clock_summary
    assert clock_summary([0] * 8) == {}
    s = clock_summary([10, 5, 1, 1, 300, 100, 3, 1])
    assert s["encrypt"]["clock_ghz"] == pytest.approx(0.2)      # 2 cycles per 10 ns tick
    assert s["decrypt"]["cycles_per_launch"] == pytest.approx(100.0)
    assert s["decrypt"]["wg_span_ms"] == pytest.approx(100 / 3 / 1e5)
