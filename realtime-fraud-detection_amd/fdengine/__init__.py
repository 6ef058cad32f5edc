"""fdengine — MI355X-native drop-in for the fraud-scoring hot path of
AjayAlluri/realtime-fraud-detection (windowed features -> XGBoost + IsolationForest -> blend).

Host side of libfdengine.so (HIP/gfx950, C-ABI in include/fdengine.h). Importing this package
loads the native library and fails loudly if it is missing: there is no CPU fallback.
"""
from . import _native  # noqa: F401  (loads libfdengine.so or raises ImportError)
from .engine import FraudEngine, device_count, pack_forest_host  # noqa: F401
from .forest import (ForestArrays, UnsupportedModel, iforest_from_sklearn,  # noqa: F401
                     load_isolation_forest_joblib, load_xgboost_json, xgboost_from_json_doc)

__all__ = ["FraudEngine", "ForestArrays", "UnsupportedModel", "device_count", "iforest_from_sklearn",
           "load_isolation_forest_joblib", "load_xgboost_json", "pack_forest_host", "xgboost_from_json_doc"]
