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
