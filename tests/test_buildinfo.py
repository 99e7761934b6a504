"""Keys that tie carried PMC records to a build (bench.py roofline.traffic): library sha first, then source sha."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spark-timeseries_amd"))

from sparkts_amd.buildinfo import match_record, source_sha  # noqa: E402

W = {"series": 1048576, "T": 1024, "p": 2, "d": 1, "q": 2, "I": 1, "smear": 1}


def test_source_sha_is_stable_and_hex():
    a, b = source_sha(), source_sha()
    assert a == b and len(a) == 64 and int(a, 16) >= 0


def test_match_prefers_library_then_source_and_never_other_workloads():
    recs = [{"workload": W, "build_sha": "L1", "source_sha": "S1", "id": 1},
            {"workload": W, "build_sha": "L2", "source_sha": "S2", "id": 2},
            {"workload": dict(W, series=4096), "build_sha": "L3", "source_sha": "S3", "id": 3}]
    assert match_record(recs, W, "L2", "S1") == (recs[1], "build_sha")
    assert match_record(recs, W, "Lx", "S1") == (recs[0], "source_sha")
    assert match_record(recs, W, "L3", "S3") == (None, None)
    assert match_record(recs, W, None, None) == (None, None)
    # a record written before source keys existed matches on the library only
    assert match_record([{"workload": W, "build_sha": "L9"}], W, "Lx", None) == (None, None)
