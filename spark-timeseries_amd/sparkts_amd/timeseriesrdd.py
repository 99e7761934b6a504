"""Partition-level drop-in for `TimeSeriesRDD.mapSeries(v => Vectors.dense(ARIMA.fitModel(p,d,q,v).coefficients))`.

The reference applies the fit per record inside a Spark task (TimeSeriesRDD.scala:249-251,
python/sparkts/timeseriesrdd.py:77-93). A per-record closure cannot batch, so the drop-in works per partition
(`rdd.mapPartitions(lambda it: fit_arima_partition(it, p, d, q))`): records are bucketed by series length, each
bucket is packed into one series-major (N, T) float64 buffer and fitted by ONE call of the C ABI, and the
records come back in their original order as (key, coefficients). A failed fit yields NaN coefficients (the
reference would fail the Spark task); `with_status=True` also returns the ARIMA_ST_* code per record.
"""
import numpy as np

from .models import ARIMA as _arima


def fit_arima_partition(records, p, d, q, includeIntercept=True, method="css-cgd", userInitParams=None,
                        with_status=False, device=None):
    records = list(records)
    keys = [k for k, _ in records]
    vals = [np.asarray(v, dtype=np.float64).ravel() for _, v in records]
    out = [None] * len(records)
    by_len = {}
    for i, v in enumerate(vals):
        by_len.setdefault(len(v), []).append(i)
    for T, idx in by_len.items():
        batch = np.stack([vals[i] for i in idx]) if T > 0 else np.zeros((len(idx), 0))
        res = _arima.fit_models(p, d, q, batch, includeIntercept, method, userInitParams, device=device)
        for j, i in enumerate(idx):
            out[i] = (keys[i], res.coefficients[j].copy(), int(res.status[j]))
    for rec in out:
        yield rec if with_status else rec[:2]


def map_series_fit_arima(series_by_key, p, d, q, **kw):
    """Dict/sequence convenience: {key: series} -> {key: coefficients}."""
    items = series_by_key.items() if hasattr(series_by_key, "items") else series_by_key
    return {k: c for k, c in fit_arima_partition(items, p, d, q, **kw)}


# ---------------------------------------------------------------------------------------------------------------
# The Python <-> JVM wire format of spark-ts: one (key, series) record is
#   int32 big-endian key length | key UTF-8 bytes | int32 big-endian series length | float64 big-endian values
# (PythonConnector.scala:59-88 BytesToKeyAndSeries / KeyAndSeriesToBytes; python/sparkts/timeseriesrdd.py:239-265
# _TimeSeriesSerializer), and a stream of records is framed by pyspark's FramedSerializer (int32 big-endian frame
# length before each record). Parsing is vectorised: the values of a record are one np.frombuffer('>f8') view.
# ---------------------------------------------------------------------------------------------------------------
import struct as _struct


def key_series_to_bytes(key, vector):
    """KeyAndSeriesToBytes.call / _TimeSeriesSerializer.dumps."""
    kb = key.encode("utf-8")
    v = np.ascontiguousarray(vector, dtype=np.float64).ravel()
    return _struct.pack("!i", len(kb)) + kb + _struct.pack("!i", v.size) + v.astype(">f8").tobytes()


def bytes_to_key_series(blob):
    """BytesToKeyAndSeries.call / _TimeSeriesSerializer.loads -> (key, float64 array)."""
    mv = memoryview(blob)
    klen = _struct.unpack_from("!i", mv, 0)[0]
    key = bytes(mv[4:4 + klen]).decode("utf-8")
    n = _struct.unpack_from("!i", mv, 4 + klen)[0]
    off = 8 + klen
    if n < 0 or off + 8 * n > len(mv):
        raise ValueError("truncated (key, series) record")
    return key, np.frombuffer(mv, dtype=">f8", count=n, offset=off).astype(np.float64)


class TimeSeriesSerializer:
    """Byte-compatible with the reference's _TimeSeriesSerializer framed stream (dump_stream / load_stream)."""

    def dumps(self, obj):
        return key_series_to_bytes(*obj)

    def loads(self, blob):
        return bytes_to_key_series(blob)

    def dump_stream(self, iterator, stream):
        for obj in iterator:
            b = self.dumps(obj)
            stream.write(_struct.pack("!i", len(b)))
            stream.write(b)

    def load_stream(self, stream):
        while True:
            head = stream.read(4)
            if len(head) < 4:
                return
            (n,) = _struct.unpack("!i", head)
            yield self.loads(stream.read(n))


def fit_arima_records(blobs, p, d, q, includeIntercept=True, method="css-cgd", userInitParams=None, device=None):
    """Partition drop-in over wire-format records (what the JVM hands a Python worker): parse every
    (key, series) record, fit the partition through fit_arima_partition (one ABI call per series length), and
    return (key, coefficients) records in the same wire format (NaN coefficients for failed fits)."""
    recs = (bytes_to_key_series(b) for b in blobs)
    for key, coef in fit_arima_partition(recs, p, d, q, includeIntercept, method, userInitParams, device=device):
        yield key_series_to_bytes(key, coef)
