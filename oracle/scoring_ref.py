"""ORACLE — TEST INFRASTRUCTURE ONLY. Pure-Python restatement of EnsemblePredictor's per-model
clamp/confidence, combination strategies, decision and risk level
(reference: services/ml-models/src/models/ensemble_predictor.py).

Evaluated with Python floats in the reference's order, so it reproduces the reference bit for bit;
pinned against the imported reference by tests/golden/ensemble_cases.json.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

# ensemble_predictor.py:331-337
CONF_MULT = {"xgboost_primary": 1.0, "lstm_sequential": 0.8, "bert_text": 0.7, "graph_neural": 0.6,
             "isolation_forest": 0.5}
DECISIONS = ("APPROVE", "REVIEW", "DECLINE", "APPROVE_WITH_MONITORING")
RISKS = ("VERY_LOW", "LOW", "MEDIUM", "HIGH", "CRITICAL")


def clamp_prob(p) -> float:
    """_predict_single_model :203 — max(0.0, min(1.0, fraud_prob))."""
    return max(0.0, min(1.0, float(p)))


def model_confidence(p: float, name: str) -> float:
    """_calculate_model_confidence :325-342."""
    distance = abs(p - 0.5)
    mult = CONF_MULT.get(name, 0.5)
    return min(1.0, distance * 2 * mult)


def normalized_weights(weights: Dict[str, float]) -> Dict[str, float]:
    """_get_model_weights :62-73 (weights of ENABLED models)."""
    total = sum(weights.values())
    if total > 0:
        return {k: w / total for k, w in weights.items()}
    return dict(weights)


def weighted_average(preds: List[Tuple[str, float, float]], w: Dict[str, float]):
    """:263-284. preds: [(name, prediction, confidence)] in model order."""
    total_weight = 0.0
    weighted_sum = 0.0
    confidence_sum = 0.0
    for name, p, c in preds:
        weight = w.get(name, 0.0)
        weighted_sum += p * weight
        confidence_sum += c * weight
        total_weight += weight
    if total_weight == 0:
        return 0.5, 0.0
    return weighted_sum / total_weight, confidence_sum / total_weight


def voting(preds, fraud_threshold: float):
    """:286-303."""
    fraud_votes = 0
    total = len(preds)
    cs = 0.0
    for _, p, c in preds:
        if p > fraud_threshold:
            fraud_votes += 1
        cs += c
    return (fraud_votes / total if total > 0 else 0.0), (cs / total if total > 0 else 0.0)


def stacking(preds, w):
    """:305-323."""
    tc = sum(c for _, _, c in preds)
    if tc == 0:
        return weighted_average(preds, w)
    ws = sum(p * c for _, p, c in preds)
    return ws / tc, tc / len(preds)


def decision(fp: float, conf: float, confidence_threshold: float = 0.7) -> str:
    """:344-356."""
    if conf < confidence_threshold:
        return "REVIEW"
    if fp >= 0.95:
        return "DECLINE"
    elif fp >= 0.8:
        return "REVIEW"
    elif fp >= 0.6:
        return "APPROVE_WITH_MONITORING"
    return "APPROVE"


def risk_level(fp: float) -> str:
    """:358-369."""
    if fp >= 0.95:
        return "CRITICAL"
    elif fp >= 0.8:
        return "HIGH"
    elif fp >= 0.6:
        return "MEDIUM"
    elif fp >= 0.3:
        return "LOW"
    return "VERY_LOW"


def blend_row(names: Sequence[str], probs: Sequence[Optional[float]], weights: Dict[str, float],
              strategy: str = "weighted_average", fraud_threshold: float = 0.5,
              confidence_threshold: float = 0.7):
    """One transaction: probs[i] None = model i failed (dropped, :175-181).
    -> (fraud_probability, confidence, decision, risk_level)."""
    preds = []
    for name, p in zip(names, probs):
        if p is None:
            continue
        q = clamp_prob(p)
        preds.append((name, q, model_confidence(q, name)))
    if not preds:
        raise ValueError("No model predictions available")
    if strategy == "weighted_average":
        fp, conf = weighted_average(preds, weights)
    elif strategy == "voting":
        fp, conf = voting(preds, fraud_threshold)
    elif strategy == "stacking":
        fp, conf = stacking(preds, weights)
    else:
        raise ValueError(f"Unknown ensemble strategy: {strategy}")
    return fp, conf, decision(fp, conf, confidence_threshold), risk_level(fp)
