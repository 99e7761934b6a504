"""Parity of the exact configuration bench.py times: fit_pipeline 6 on GPU_MAX_HW_QUEUES=8.

With P > 1 contexts the fit kernel's drained bulk workgroups exit instead of turning express, and up to P fits run
concurrently on separate hardware queues -- a different schedule from the serial fit the other parity tests use. The
queue count must be set before HIP initialises, so a fresh child process (tests/_pipeline_child.py, started as a
child, never exec'd) runs 8 consecutive C2 fits of 65 536 series over 6 contexts and compares every output set with
a serial fit of the same batch bit for bit; this test then checks the serial result's first rows against the oracle.
Reference: ARIMA.fitModel (ARIMA.scala:79-116) per series, whatever the schedule.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bench_configuration_pipeline6_queues8_matches_serial(tmp_path):
    out = str(tmp_path / "pipe.npz")
    env = dict(os.environ, GPU_MAX_HW_QUEUES="8", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, os.path.join(ROOT, "tests", "_pipeline_child.py"), "--N", "65536", "--pipeline", "6",
           "--fits", "8", "--out", out]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    z = np.load(out, allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    assert meta["hw_queues"] == "8"
    assert meta["serial_done"] == 65536 and meta["last_done"] == 65536, meta
    assert meta["mismatch_per_set"] == [0] * 6, meta
    # the serial fit itself against the oracle (first 256 rows)
    s = z["series"]
    st, coef, ll, cnt = O.fit_batch(s, 2, 1, 2, 1)
    assert np.array_equal(z["status"], st)
    assert np.array_equal(z["n_eval"], cnt[:, 0]) and np.array_equal(z["n_grad"], cnt[:, 1])
    ok = st == 0
    assert np.array_equal(z["coef"][ok].view(np.int64), coef[ok].view(np.int64))
    assert np.array_equal(z["ll"][ok].view(np.int64), ll[ok].view(np.int64))
