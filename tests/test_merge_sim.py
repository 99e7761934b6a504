"""k_cg_fit's drain-merge protocol (spark-timeseries_amd/csrc/arima_kernels_impl.hpp, "Drain merge") restated on host
threads (tests/sim/merge_sim.cpp): every series finished exactly once, every wave leaves, the pool never
overflows -- across wave counts, thresholds (up to 64: every drained wave offers its slots), a pool small enough to
fill, and under ThreadSanitizer for the entry / ready-word ordering. The GPU side of the same property is
tests/test_gpu_parity.py::test_drain_merge_is_transparent."""
import os
import subprocess

import pytest

SIM = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sim")
BUILD = os.path.join(SIM, "_build")


def _build(name, flags):
    os.makedirs(BUILD, exist_ok=True)
    out = os.path.join(BUILD, name)
    src = os.path.join(SIM, "merge_sim.cpp")
    if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
        subprocess.check_call(["g++", "-std=c++17", "-pthread", "-Wall", *flags, "-o", out, src])
    return out


CASES = [(8, 5000, 16, 1, 24576), (64, 50000, 16, 2, 24576), (256, 200000, 64, 3, 24576), (128, 100000, 64, 4, 200),
         (128, 100000, 1, 5, 24576), (3, 2000, 16, 6, 24576)]


@pytest.mark.parametrize("waves,series,threshold,seed,cap", CASES)
def test_merge_protocol(waves, series, threshold, seed, cap):
    exe = _build("merge_sim", ["-O2"])
    r = subprocess.run([exe, str(waves), str(series), str(threshold), str(seed), str(cap)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "lost 0, finished twice 0" in r.stdout


def test_merge_protocol_thread_sanitizer():
    exe = _build("merge_sim_tsan", ["-O1", "-g", "-fsanitize=thread"])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    for args in [(32, 20000, 16, 7, 24576), (16, 10000, 64, 8, 100)]:
        r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "WARNING: ThreadSanitizer" not in r.stderr
