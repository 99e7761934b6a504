from . import ARIMA  # noqa: F401
