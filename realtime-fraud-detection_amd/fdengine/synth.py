"""Seeded synthetic inputs and model files (no network: no datasets, no pretrained models).

* `feature_matrix`: a scoring-vector-shaped f32 matrix (counts, ratios, flags, scores; clipped to
  +-10 like EnsemblePredictor._prepare_features, ml/models/ensemble_predictor.py:248) for the
  XGBoost-only bench (BASELINE config 2: 500 trees, depth 8, 50 features).
* `xgboost_doc`: a binary:logistic gbtree model in the XGBoost 2.0.3 JSON schema (the file format
  ml/models/model_manager.py:157-161 loads). Split thresholds are values drawn from the data, so
  ties x == threshold occur and exercise the `x < thr` convention.
* `isolation_forest`: sklearn IsolationForest trained with the reference trainer's recipe
  (ml/training/model_trainer.py:246-251: contamination=0.05, n_estimators=100, random_state=42).
"""
from __future__ import annotations

import json
from typing import Optional

import numpy as np


def feature_matrix(n: int, n_features: int, seed: int = 42, nan_frac: float = 0.0) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    cols = []
    for j in range(n_features):
        kind = j % 5
        if kind == 0:
            c = rng.poisson(3.0, n).astype(np.float64)                 # counts
        elif kind == 1:
            c = rng.lognormal(0.0, 1.0, n)                             # ratios / amounts
        elif kind == 2:
            c = (rng.random(n) < 0.2).astype(np.float64)               # flags
        elif kind == 3:
            c = rng.beta(2.0, 8.0, n)                                  # risk scores
        else:
            c = rng.integers(0, 24, n).astype(np.float64)              # hour-like
        cols.append(c)
    X = np.clip(np.stack(cols, axis=1), -10.0, 10.0).astype(np.float32)
    if nan_frac > 0:
        X[rng.random(X.shape) < nan_frac] = np.nan
    return np.ascontiguousarray(X)


def xgboost_doc(n_trees: int, depth: int, n_features: int, X_ref: np.ndarray, seed: int = 7,
                p_leaf: float = 0.0, base_score: float = 0.5, num_feature: Optional[int] = None) -> dict:
    """Random gbtree trees in the XGBoost 2.0.3 JSON schema. p_leaf: chance a node at depth >= 2
    stops early (ragged trees exercise the perfect-tree padding)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    X_ref = np.asarray(X_ref, dtype=np.float32)
    trees = []
    for tid in range(n_trees):
        left, right, parent, feat, cond, dleft, depthv = [], [], [], [], [], [], []

        def new(par, d):
            left.append(-1); right.append(-1); parent.append(par); feat.append(0)
            cond.append(0.0); dleft.append(0); depthv.append(d)
            return len(left) - 1

        new(2147483647, 0)
        q = 0
        while q < len(left):  # breadth-first expansion: XGBoost's depthwise node numbering
            d = depthv[q]
            if d < depth and not (d >= 2 and rng.random() < p_leaf):
                f = int(rng.integers(0, n_features))
                col = X_ref[:, f]
                col = col[~np.isnan(col)]
                thr = float(col[rng.integers(0, len(col))]) if len(col) else 0.0
                feat[q] = f
                cond[q] = float(np.float32(thr))
                dleft[q] = int(rng.integers(0, 2))
                left[q] = new(q, d + 1)
                right[q] = new(q, d + 1)
            else:
                cond[q] = float(np.float32(rng.normal(0.0, 0.1)))
            q += 1
        m = len(left)
        trees.append({
            "base_weights": [float(c) for c in cond],
            "categories": [], "categories_nodes": [], "categories_segments": [], "categories_sizes": [],
            "default_left": dleft, "id": tid, "left_children": left,
            "loss_changes": [0.0 if l == -1 else 1.0 for l in left], "parents": parent,
            "right_children": right, "split_conditions": cond, "split_indices": feat,
            "split_type": [0] * m, "sum_hessian": [1.0] * m,
            "tree_param": {"num_deleted": "0", "num_feature": str(num_feature or n_features),
                           "num_nodes": str(m), "size_leaf_vector": "1"},
        })
    nf = num_feature or n_features
    return {
        "learner": {
            "attributes": {}, "feature_names": [], "feature_types": [],
            "gradient_booster": {
                "model": {
                    "gbtree_model_param": {"num_parallel_tree": "1", "num_trees": str(n_trees)},
                    "iteration_indptr": list(range(n_trees + 1)),
                    "tree_info": [0] * n_trees,
                    "trees": trees,
                },
                "name": "gbtree",
            },
            "learner_model_param": {"base_score": f"{base_score:E}", "boost_from_average": "1",
                                    "num_class": "0", "num_feature": str(nf), "num_target": "1"},
            "objective": {"name": "binary:logistic", "reg_loss_param": {"scale_pos_weight": "1"}},
        },
        "version": [2, 0, 3],
    }


def write_xgboost_json(path: str, doc: dict) -> None:
    with open(path, "w") as f:
        json.dump(doc, f)


def isolation_forest(X_train: np.ndarray, n_estimators: int = 100, contamination: float = 0.05,
                     random_state: int = 42):
    from sklearn.ensemble import IsolationForest
    m = IsolationForest(contamination=contamination, n_estimators=n_estimators, random_state=random_state)
    m.fit(X_train)
    return m
