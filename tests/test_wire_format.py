"""The spark-ts Python <-> JVM (key, series) wire format (PythonConnector.scala:59-88,
python/sparkts/timeseriesrdd.py:239-265): the reference's own serializer test (test_timeseriesrdd.py:11-22) restated,
plus byte-level layout checks against a hand-built big-endian record. CPU only."""
import struct
from io import BytesIO

import numpy as np

from sparkts_amd.timeseriesrdd import TimeSeriesSerializer, bytes_to_key_series, key_series_to_bytes


def test_times_series_serializer_roundtrip():
    # test_timeseriesrdd.py:11-22
    serializer = TimeSeriesSerializer()
    stream = BytesIO()
    series = [('abc', np.array([4.0, 4.0, 5.0])), ('123', np.array([1.0, 2.0, 3.0]))]
    serializer.dump_stream(iter(series), stream)
    stream.seek(0)
    back = list(serializer.load_stream(stream))
    assert back[0][0] == series[0][0] and back[1][0] == series[1][0]
    assert (back[0][1] == series[0][1]).all() and (back[1][1] == series[1][1]).all()


def test_record_layout_is_big_endian_length_prefixed():
    # KeyAndSeriesToBytes: putInt(keyLen) put(key) putInt(size) putDouble(v)... (java.nio.ByteBuffer: big-endian)
    key, vec = "sér-1", np.array([1.5, -0.0, np.nan, 1e300])
    kb = key.encode("utf-8")
    ref = struct.pack(">i", len(kb)) + kb + struct.pack(">i", 4) + b"".join(struct.pack(">d", v) for v in vec)
    assert key_series_to_bytes(key, vec) == ref
    k2, v2 = bytes_to_key_series(ref)
    assert k2 == key and np.array_equal(v2.view(np.int64), vec.view(np.int64))


def test_empty_series_and_key():
    b = key_series_to_bytes("", np.zeros(0))
    assert b == struct.pack(">ii", 0, 0)
    k, v = bytes_to_key_series(b)
    assert k == "" and v.size == 0
