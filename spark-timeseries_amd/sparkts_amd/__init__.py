"""sparkts_amd — MI355X-native drop-in for spark-ts's ARIMA CSS-CGD fit path (ARIMA.fitModel under mapSeries).

Host-side mirror of the reference's Python API (python/sparkts/) over the C ABI of libsparkts_arima.so.
"""
from . import _lib  # noqa: F401
from .models import ARIMA  # noqa: F401
from .timeseriesrdd import fit_arima_partition, map_series_fit_arima  # noqa: F401

__version__ = "0.1.0"
