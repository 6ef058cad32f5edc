"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference algorithms on the hot path, used as the checker by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg. Nothing under
realtime-fraud-detection_amd/ imports this package; the product path has no CPU fallback.

  oracle_forest.c    XGBoost 2.0.3 gbtree predict + sklearn IsolationForest scoring (C, OpenMP)
  oracle_features.c  card-velocity state + feature vector restatement (C)
  scoring_ref.py     pure-Python restatement of EnsemblePredictor blend/decision (f64, ref order)
  features_ref.py    pure-Python restatement of FeatureProcessor + _prepare_features
  forest_ref.py      pure-Python XGBoost / IF walkers (small cases; cross-checks the C restatement)

Parity status (see DESIGN.md "Oracle"): FeatureProcessor/_prepare_features, the blend and the
IsolationForest are pinned by golden vectors produced by importing the reference Python and
sklearn in the build container (tests/golden/make_golden.py). XGBoost is parity-unpinned against
the library (xgboost is not installable offline); it is pinned by known-answer trees. The Java
velocity/feature semantics are parity-unpinned (no JDK, no tests in the reference).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
# FD_ORACLE_LIB: another build of the same sources (the sanitizer build of tests/test_oracle_sanitizers.py)
LIB_PATH = Path(os.environ.get("FD_ORACLE_LIB") or ORACLE_DIR / "build" / "liboracle.so")

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            import importlib.util
            spec = importlib.util.spec_from_file_location(
                "fdengine_build", ORACLE_DIR.parent / "realtime-fraud-detection_amd" / "fdengine" / "build.py")
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            mod.build_oracle()
        L = C.CDLL(str(LIB_PATH))
        vp, i32, i64, d = C.c_void_p, C.c_int32, C.c_int64, C.c_double
        L.orc_xgb_predict.restype = C.c_int
        L.orc_xgb_predict.argtypes = [i64, i32, vp, i32, vp, vp, vp, vp, vp, vp, vp, d, i32, vp, vp, vp]
        L.orc_iforest_predict.restype = C.c_int
        L.orc_iforest_predict.argtypes = [i64, i32, vp, i32, vp, vp, vp, vp, vp, vp, vp, d, d, i32, vp, vp, vp]
        L.orc_blend_weighted.restype = C.c_int
        L.orc_blend_weighted.argtypes = [i64, i32, vp, vp, vp, d, i32, vp, vp, vp, vp]
        L.orc_xgb_base_margin.restype = C.c_float
        L.orc_xgb_base_margin.argtypes = [d]
        _register_features(L)
        _lib = L
    return _lib


def _register_features(L) -> None:
    from . import features_c
    features_c.register(L)


def _ptr(a):
    return None if a is None else a.ctypes.data


def _forest_arrays(fa):
    return dict(offs=np.ascontiguousarray(fa.offsets, np.int64), left=np.ascontiguousarray(fa.left, np.int32),
                right=np.ascontiguousarray(fa.right, np.int32), feat=np.ascontiguousarray(fa.feature, np.int32),
                thr=np.ascontiguousarray(fa.threshold, np.float64),
                dl=np.ascontiguousarray(fa.default_left, np.uint8),
                lv=np.ascontiguousarray(fa.leaf_value, np.float64))


def xgb_predict(fa, X: np.ndarray, nthreads: int = 0, want_leaf: bool = False):
    """-> (prob f32 [n], margin f32 [n], leaf int32 [n, T] or None)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    n, ld = X.shape
    a = _forest_arrays(fa)
    T = fa.n_trees
    margin = np.empty(n, np.float32)
    prob = np.empty(n, np.float32)
    leaf = np.empty((n, T), np.int32) if want_leaf else None
    lib().orc_xgb_predict(n, ld, _ptr(X), T, _ptr(a["offs"]), _ptr(a["left"]), _ptr(a["right"]), _ptr(a["feat"]),
                          _ptr(a["thr"]), _ptr(a["dl"]), _ptr(a["lv"]), float(fa.base_score), nthreads,
                          _ptr(margin), _ptr(prob), _ptr(leaf))
    return prob, margin, leaf


def iforest_predict(fa, X: np.ndarray, nthreads: int = 0, want_leaf: bool = False):
    """-> (prob f64 [n], depth-sum f64 [n], leaf int32 [n, T] or None)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    n, ld = X.shape
    a = _forest_arrays(fa)
    T = fa.n_trees
    depth = np.empty(n, np.float64)
    prob = np.empty(n, np.float64)
    leaf = np.empty((n, T), np.int32) if want_leaf else None
    lib().orc_iforest_predict(n, ld, _ptr(X), T, _ptr(a["offs"]), _ptr(a["left"]), _ptr(a["right"]),
                              _ptr(a["feat"]), _ptr(a["thr"]), _ptr(a["dl"]), _ptr(a["lv"]), float(fa.if_offset),
                              float(fa.if_denominator), nthreads, _ptr(depth), _ptr(prob), _ptr(leaf))
    return prob, depth, leaf


def blend_weighted(probs: np.ndarray, weights, mults, confidence_threshold=0.7, nthreads: int = 0):
    """CPU-baseline blend (weighted average), probs [M, n] -> (fp, conf, decision, risk)."""
    P = np.ascontiguousarray(probs, np.float64)
    M, n = P.shape
    w = np.ascontiguousarray(weights, np.float64)
    m = np.ascontiguousarray(mults, np.float64)
    fp, conf = np.empty(n), np.empty(n)
    dec, risk = np.empty(n, np.uint8), np.empty(n, np.uint8)
    lib().orc_blend_weighted(n, M, _ptr(P), _ptr(w), _ptr(m), float(confidence_threshold), nthreads, _ptr(fp),
                             _ptr(conf), _ptr(dec), _ptr(risk))
    return fp, conf, dec, risk
