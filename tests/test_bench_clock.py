"""bench.py's roofline.clock: the rocm-smi sampler parses this image's output
format, picks this rank's GPU, and degrades to None without rocm-smi."""
import subprocess
import time

import bench

SMI = """
============================ ROCm System Management Interface ============================
GPU[0]		: sclk clock level: 1: (2079Mhz)
GPU[0]		: Current Socket Graphics Package Power (W): 1339.0
GPU[1]		: sclk clock level: 1: (1500Mhz)
GPU[1]		: Current Socket Graphics Package Power (W): 900.0
==========================================================================================
"""


class _Done:
    stdout = SMI


def _sample(monkeypatch, local, fake):
    monkeypatch.setattr(subprocess, 'run', fake)
    monkeypatch.delenv('ROCR_VISIBLE_DEVICES', raising=False)
    monkeypatch.delenv('HIP_VISIBLE_DEVICES', raising=False)
    c = bench.ClockSampler(local)
    c.start()
    time.sleep(0.35)
    return c.stop()


def test_sampler_parses_rocm_smi(monkeypatch):
    r = _sample(monkeypatch, 0, lambda *a, **k: _Done())
    assert r['samples'] >= 1 and r['sclk_mhz_median'] == 2079 and r['power_w_median'] == 1339.0
    r = _sample(monkeypatch, 1, lambda *a, **k: _Done())
    assert r['sclk_mhz_median'] == 1500 and r['power_w_median'] == 900.0


def test_sampler_without_rocm_smi(monkeypatch):
    def missing(*a, **k):
        raise FileNotFoundError('rocm-smi')
    assert _sample(monkeypatch, 0, missing) is None


def test_held_clock_fraction():
    h = bench.held_clock({'sclk_mhz_median': 2080, 'power_w_median': 1340.0, 'samples': 5}, 1369.0, 2500.0)
    assert abs(h['peak_at_held_clock'] - 2500.0 * 2080 / 2400) < 0.1
    assert abs(h['frac_at_held_clock'] - 1369.0 / (2500.0 * 2080 / 2400)) < 1e-4
    assert bench.held_clock(None, 1.0, 2.0) is None
    short = bench.held_clock({'sclk_mhz_median': 2384, 'power_w_median': 351.0, 'samples': 1}, 1369.0, 2500.0)
    assert 'frac_at_held_clock' not in short and 'note' in short
