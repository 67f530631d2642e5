"""Validation / test metrics on device."""
from .regression_accuracy import RegressionAccuracy  # noqa: F401
from .sr_metrics import METRIC_KEYS, SRMetrics  # noqa: F401
