import glob
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "spark-timeseries_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")


def load_case(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    arr = {k: z[k] for k in z.files if k != "meta"}
    return meta, arr


def all_cases(prefix=""):
    """Golden fit fixtures (prefix ""), or those of a prefix; the autoFit fixtures (autofit_*) hold another layout
    and are only listed when asked for by their prefix."""
    names = sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))
    return names if prefix.startswith("autofit") else [n for n in names if not n.startswith("autofit_")]


@pytest.fixture(scope="session")
def engine():
    import sparkts_amd._lib as L
    return L.Engine.get(0)
