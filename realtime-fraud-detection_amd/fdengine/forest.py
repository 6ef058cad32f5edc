"""Model-file formats on the path, read unchanged, flattened to the engine's original-tree arrays.

* XGBoost 2.0.3 JSON (`XGBClassifier.save_model(".../xgboost/fraud_classifier.json")`,
  reference ml/training/model_trainer.py:95-108; loaded by ml/models/model_manager.py:157-161).
  Schema: learner.gradient_booster.model.trees[i].{left_children, right_children, split_indices,
  split_conditions, default_left, split_type}; a node is a leaf when left_children[i] == -1 and its
  leaf weight is split_conditions[i]; learner.learner_model_param.{base_score, num_feature,
  num_class}; learner.objective.name.
* scikit-learn IsolationForest pickled with joblib (ml/training/model_trainer.py:246-266; loaded by
  ml/models/model_manager.py:197-200). The host unpickles it with sklearn exactly as the reference
  does, then passes tree_.{children_left, children_right, feature, threshold, missing_go_to_left}
  and the per-node path-length terms sklearn itself adds in `_compute_score_samples`.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import numpy as np

from . import _native as N


class UnsupportedModel(ValueError):
    pass


@dataclass
class ForestArrays:
    """Original trees, concatenated (CSR by `offsets`). Mirrors fd_tree_arrays."""
    kind: int
    num_feature: int
    offsets: np.ndarray          # int64 [T+1]
    left: np.ndarray             # int32
    right: np.ndarray            # int32
    feature: np.ndarray          # int32
    threshold: np.ndarray        # float64
    default_left: np.ndarray     # uint8
    leaf_value: np.ndarray       # float64
    base_score: float = 0.5
    if_offset: float = 0.0
    if_denominator: float = 0.0
    meta: Dict[str, Any] = field(default_factory=dict)

    @property
    def n_trees(self) -> int:
        return len(self.offsets) - 1

    def c_structs(self):
        """(fd_forest_params, fd_tree_arrays, keepalive) for the C-ABI."""
        arrs = dict(
            offsets=np.ascontiguousarray(self.offsets, dtype=np.int64),
            left=np.ascontiguousarray(self.left, dtype=np.int32),
            right=np.ascontiguousarray(self.right, dtype=np.int32),
            feature=np.ascontiguousarray(self.feature, dtype=np.int32),
            threshold=np.ascontiguousarray(self.threshold, dtype=np.float64),
            default_left=np.ascontiguousarray(self.default_left, dtype=np.uint8),
            leaf_value=np.ascontiguousarray(self.leaf_value, dtype=np.float64),
        )
        import ctypes as C

        def P(a, t):
            return a.ctypes.data_as(C.POINTER(t))

        t = N.fd_tree_arrays(
            self.n_trees, P(arrs["offsets"], C.c_int64), P(arrs["left"], C.c_int32), P(arrs["right"], C.c_int32),
            P(arrs["feature"], C.c_int32), P(arrs["threshold"], C.c_double), P(arrs["default_left"], C.c_uint8),
            P(arrs["leaf_value"], C.c_double))
        p = N.fd_forest_params(self.kind, self.num_feature, float(self.base_score), float(self.if_offset),
                               float(self.if_denominator))
        return p, t, arrs


def _concat(trees: List[Dict[str, np.ndarray]], kind: int, num_feature: int, **kw) -> ForestArrays:
    sizes = [len(t["left"]) for t in trees]
    offsets = np.zeros(len(trees) + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(sizes)

    def cat(k, dt):
        return np.concatenate([np.asarray(t[k], dtype=dt) for t in trees]) if trees else np.zeros(0, dt)

    return ForestArrays(kind=kind, num_feature=num_feature, offsets=offsets, left=cat("left", np.int32),
                        right=cat("right", np.int32), feature=cat("feature", np.int32),
                        threshold=cat("threshold", np.float64), default_left=cat("default_left", np.uint8),
                        leaf_value=cat("leaf_value", np.float64), **kw)


# ----------------------------------------------------------------------------------------- XGBoost

def xgboost_from_json_doc(doc: Dict[str, Any]) -> ForestArrays:
    learner = doc["learner"]
    obj = learner.get("objective", {}).get("name")
    if obj != "binary:logistic":
        raise UnsupportedModel(f"objective {obj!r} not supported (binary:logistic only)")
    gb = learner["gradient_booster"]
    if gb.get("name") != "gbtree":
        raise UnsupportedModel(f"booster {gb.get('name')!r} not supported (gbtree only)")
    lmp = learner["learner_model_param"]
    if int(float(lmp.get("num_class", "0"))) > 1:
        raise UnsupportedModel("multi-class models are not supported")
    num_feature = int(float(lmp["num_feature"]))
    base_score = float(lmp["base_score"])
    model = gb["model"]
    trees = []
    for tr in model["trees"]:
        left = np.asarray(tr["left_children"], dtype=np.int64)
        st = tr.get("split_type")
        if st is not None and np.any(np.asarray(st) != 0):
            raise UnsupportedModel("categorical splits are not supported")
        tp = tr.get("tree_param", {})
        if int(float(tp.get("size_leaf_vector", "1"))) > 1:
            raise UnsupportedModel("vector leaves are not supported")
        leaf = left == -1
        cond = np.asarray(tr["split_conditions"], dtype=np.float64)
        feat = np.where(leaf, 0, np.asarray(tr["split_indices"], dtype=np.int64))
        trees.append(dict(
            left=np.where(leaf, -1, left), right=np.asarray(tr["right_children"], dtype=np.int64),
            feature=feat, threshold=np.where(leaf, 0.0, cond),
            default_left=np.asarray(tr["default_left"], dtype=np.uint8),
            # XGBoost holds node values as f32; JSON prints them round-trip exact
            leaf_value=np.where(leaf, cond.astype(np.float32).astype(np.float64), 0.0)))
    return _concat(trees, N.FD_FOREST_XGB_BINARY_LOGISTIC, num_feature, base_score=base_score,
                   meta={"n_trees": len(trees)})


def load_xgboost_json(path: str) -> ForestArrays:
    with open(path, "r") as f:
        return xgboost_from_json_doc(json.load(f))


# ----------------------------------------------------------------------------------- IsolationForest

def iforest_from_sklearn(model) -> ForestArrays:
    """Flatten a fitted sklearn IsolationForest (sklearn/ensemble/_iforest.py)."""
    from sklearn.ensemble._iforest import _average_path_length

    n_features = int(model.n_features_in_)
    subsample = int(model._max_features) != n_features
    trees = []
    for i, (est, feats) in enumerate(zip(model.estimators_, model.estimators_features_)):
        t = est.tree_
        left = np.asarray(t.children_left, dtype=np.int64)
        leaf = left == -1
        f = np.asarray(t.feature, dtype=np.int64)
        if subsample:
            f = np.where(leaf, 0, np.asarray(feats, dtype=np.int64)[np.where(leaf, 0, f)])
        else:
            f = np.where(leaf, 0, f)
        dl = getattr(t, "missing_go_to_left", None)
        dl = np.zeros(len(left), np.uint8) if dl is None else np.asarray(dl, dtype=np.uint8)
        # exactly the per-leaf term _parallel_compute_tree_depths adds: (dpl + apl) - 1.0, f64
        lv = (np.asarray(model._decision_path_lengths[i], dtype=np.float64)
              + np.asarray(model._average_path_length_per_tree[i], dtype=np.float64) - 1.0)
        trees.append(dict(left=np.where(leaf, -1, left), right=np.asarray(t.children_right, dtype=np.int64),
                          feature=f, threshold=np.where(leaf, 0.0, np.asarray(t.threshold, dtype=np.float64)),
                          default_left=dl, leaf_value=np.where(leaf, lv, 0.0)))
    max_samples = getattr(model, "_max_samples", model.max_samples_)
    denom = float(len(model.estimators_) * _average_path_length([max_samples])[0])
    return _concat(trees, N.FD_FOREST_SKLEARN_IFOREST, n_features, if_offset=float(model.offset_),
                   if_denominator=denom, meta={"n_trees": len(trees)})


def load_isolation_forest_joblib(path: str) -> ForestArrays:
    import joblib
    return iforest_from_sklearn(joblib.load(path))
