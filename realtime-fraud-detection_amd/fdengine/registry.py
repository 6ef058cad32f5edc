"""Model registry + ensemble settings for the scoring path.

The reference keeps these on `utils.config.Config` (services/ml-models/src/utils/config.py:9-27,
126-219). The engine accepts that object unchanged (duck-typed: `.models` dict of ModelConfig with
name/model_type/model_path/weight/enabled, `.ensemble` with strategy/confidence_threshold/
fraud_threshold/enable_explanation, `.get_enabled_models()`, `.get_model_config()`).
`ScoringConfig` below is a minimal stand-alone equivalent of just those members, so the engine and
its tests run where the reference's service code is absent (the GPU box).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Any, Dict, List


@dataclass
class ModelConfig:
    name: str
    model_type: str          # 'xgboost' | 'tensorflow' | 'pytorch' | 'transformers' | 'sklearn'
    model_path: str
    weight: float = 1.0
    enabled: bool = True
    preprocessing_steps: List[str] = field(default_factory=list)
    hyperparameters: Dict[str, Any] = field(default_factory=dict)


@dataclass
class EnsembleConfig:
    strategy: str = "weighted_average"
    confidence_threshold: float = 0.7
    fraud_threshold: float = 0.5
    enable_explanation: bool = True


# (name, type, relative path, weight) in the reference's registry order (config.py:128-199)
_REGISTRY = (
    ("xgboost_primary", "xgboost", ("xgboost", "fraud_classifier.json"), 0.4),
    ("lstm_sequential", "tensorflow", ("tensorflow", "lstm_fraud_model.h5"), 0.25),
    ("bert_text", "transformers", ("transformers", "distilbert-fraud"), 0.15),
    ("graph_neural", "pytorch", ("pytorch", "gnn_fraud_model.pth"), 0.15),
    ("isolation_forest", "sklearn", ("sklearn", "isolation_forest.joblib"), 0.05),
)


class ScoringConfig:
    def __init__(self, models_base_path: str = None):
        base = models_base_path or os.getenv("MODELS_PATH", "/app/models")
        self.models_base_path = base
        self.models: Dict[str, ModelConfig] = {
            name: ModelConfig(name=name, model_type=mt, model_path=os.path.join(base, *rel), weight=w)
            for name, mt, rel, w in _REGISTRY
        }
        env = os.getenv
        self.ensemble = EnsembleConfig(
            strategy=env("ENSEMBLE_STRATEGY", "weighted_average"),
            confidence_threshold=float(env("CONFIDENCE_THRESHOLD", "0.7")),
            fraud_threshold=float(env("FRAUD_THRESHOLD", "0.5")),
            enable_explanation=env("ENABLE_EXPLANATION", "true").lower() == "true")

    def get_model_config(self, name: str) -> ModelConfig:
        if name not in self.models:
            raise ValueError(f"Model '{name}' not found in configuration")
        return self.models[name]

    def get_enabled_models(self) -> Dict[str, ModelConfig]:
        return {n: c for n, c in self.models.items() if c.enabled}

    def disable_model(self, name: str) -> None:
        if name in self.models:
            self.models[name].enabled = False

    def enable_model(self, name: str) -> None:
        if name in self.models:
            self.models[name].enabled = True

    def update_model_weight(self, name: str, weight: float) -> None:
        if name in self.models:
            self.models[name].weight = weight
