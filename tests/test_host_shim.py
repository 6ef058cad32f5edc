"""CPU: host-side logic of the drop-in (no device calls).

* fdengine.ensemble.prepare_features reproduces the reference's _prepare_features vectors
  (golden, generated from the reference itself).
* the registry mirrors the reference's model set/order/weights.
"""
import asyncio
import json

import numpy as np

from conftest import GOLDEN
from oracle import features_ref as FR


def test_prepare_features_matches_reference_golden():
    from fdengine.ensemble import prepare_features, prepare_matrix
    cases = [c for c in json.loads((GOLDEN / "feature_processor_cases.json").read_text()) if "vector" in c]
    processed = [FR.process_features(c["raw"]) for c in cases]
    for c, p in zip(cases, processed):
        np.testing.assert_array_equal(prepare_features(p)[0], np.array(c["vector"]))
    X = prepare_matrix(processed)
    np.testing.assert_array_equal(X, np.array([c["vector"] for c in cases]))


def test_registry_mirrors_reference_order_and_weights():
    from fdengine.registry import ScoringConfig
    cfg = ScoringConfig("/models")
    assert list(cfg.models) == ["xgboost_primary", "lstm_sequential", "bert_text", "graph_neural", "isolation_forest"]
    assert [cfg.models[n].weight for n in cfg.models] == [0.4, 0.25, 0.15, 0.15, 0.05]
    assert cfg.models["xgboost_primary"].model_path == "/models/xgboost/fraud_classifier.json"
    assert cfg.models["isolation_forest"].model_path == "/models/sklearn/isolation_forest.joblib"
    cfg.disable_model("bert_text")
    assert "bert_text" not in cfg.get_enabled_models()
