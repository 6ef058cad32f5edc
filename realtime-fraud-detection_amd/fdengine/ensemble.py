"""Drop-in for services/ml-models/src/models/ensemble_predictor.py (class EnsemblePredictor).

* `predict(features)` keeps the reference's per-transaction contract bit for bit: prediction cache
  (300 s / 1000 entries, :437-471), concurrent per-model calls through ModelManager.predict with
  failing models dropped (:150-183), clamp + confidence (:185-219, 325-342), weighted-average /
  voting / stacking (:252-323), decision / risk level (:344-369), explanation (:371-435).
* `predict_batch(features_list)` is the micro-batch path the reference lacks (its /batch-predict
  loops one transaction at a time, ml/main.py:235-249): one scoring-vector matrix per vector width, every
  device-resident forest scores it in one launch each, and the blend/decision/risk epilogue runs
  on the GPU (fd_score_matrix_host). Results equal per-transaction `predict` for the same inputs
  (host stand-in models aside, which are random in the reference too); the cache is bypassed.
"""
from __future__ import annotations

import asyncio
import time
from enum import Enum
from typing import Any, Dict, List, Optional

import numpy as np

from . import _native as N
from .engine import FraudEngine

_EXCLUDED = {"transaction_id", "user_id", "merchant_id", "timestamp", "currency", "payment_method", "card_type"}
_CONF_MULT = {"xgboost_primary": 1.0, "lstm_sequential": 0.8, "bert_text": 0.7, "graph_neural": 0.6,
              "isolation_forest": 0.5}
VECTOR_WIDTH = 64


class EnsembleStrategy(Enum):
    WEIGHTED_AVERAGE = "weighted_average"
    VOTING = "voting"
    STACKING = "stacking"


_STRATEGY_CODE = {EnsembleStrategy.WEIGHTED_AVERAGE: N.FD_BLEND_WEIGHTED_AVERAGE,
                  EnsembleStrategy.VOTING: N.FD_BLEND_VOTING, EnsembleStrategy.STACKING: N.FD_BLEND_STACKING}


def prepare_features(features: Dict[str, Any]) -> np.ndarray:
    """The reference's scoring-vector layout (ensemble_predictor.py:221-250): numeric values in dict
    order minus metadata keys, then the Flink `features` sub-dict's numerics, zero-padded to 64,
    clipped to [-10, 10]. -> (1, >=64) float64."""
    vals = [float(v) for k, v in features.items() if k not in _EXCLUDED and isinstance(v, (int, float))]
    sub = features.get("features")
    if isinstance(sub, dict):
        vals.extend(float(v) for v in sub.values() if isinstance(v, (int, float)))
    if len(vals) < VECTOR_WIDTH:
        vals.extend([0.0] * (VECTOR_WIDTH - len(vals)))
    return np.clip(np.array(vals).reshape(1, -1), -10, 10)


def prepare_matrix(features_list: List[Dict[str, Any]]) -> np.ndarray:
    rows = [prepare_features(f)[0] for f in features_list]
    width = max([VECTOR_WIDTH] + [len(r) for r in rows])
    X = np.zeros((len(rows), width), np.float64)
    for i, r in enumerate(rows):
        X[i, :len(r)] = r
    return X


class EnsemblePredictor:
    def __init__(self, model_manager, config):
        self.model_manager = model_manager
        self.config = config
        self.strategy = EnsembleStrategy(config.ensemble.strategy)
        self.fraud_threshold = config.ensemble.fraud_threshold
        self.confidence_threshold = config.ensemble.confidence_threshold
        self.enable_explanation = config.ensemble.enable_explanation
        self.model_weights = self._get_model_weights()
        self.prediction_cache: Dict[str, Any] = {}
        self.cache_ttl_seconds = 300

    def _get_model_weights(self) -> Dict[str, float]:
        weights = {n: c.weight for n, c in self.config.get_enabled_models().items()}
        total = sum(weights.values())
        if total > 0:
            weights = {n: w / total for n, w in weights.items()}
        return weights

    # ------------------------------------------------------------------ per-transaction (reference contract)
    async def predict(self, features: Dict[str, Any]) -> Dict[str, Any]:
        t0 = time.time()
        key = self._generate_cache_key(features)
        cached = self._get_cached_prediction(key)
        if cached:
            return cached
        X = prepare_features(features)
        preds = await self._model_predictions(X)
        if not preds:
            raise ValueError("No model predictions available")
        fp, conf = self._combine(preds)
        result = {
            "fraud_probability": fp, "fraud_score": fp, "confidence": conf,
            "risk_level": self._calculate_risk_level(fp), "decision": self._make_decision(fp, conf),
            "model_predictions": {n: p for n, p, _ in preds}, "model_confidences": {n: c for n, _, c in preds},
            "explanation": self._generate_explanation(preds, features) if self.enable_explanation else {},
            "ensemble_strategy": self.strategy.value, "processing_time_ms": (time.time() - t0) * 1000,
        }
        self._cache_prediction(key, result)
        return result

    async def _model_predictions(self, X: np.ndarray):
        enabled = [n for n in self.config.get_enabled_models() if self.model_manager.is_model_loaded(n)]
        if not enabled:
            raise ValueError("No enabled models are loaded")
        tasks = [(n, asyncio.create_task(self.model_manager.predict(n, X))) for n in enabled]
        out = []
        for name, task in tasks:
            try:
                pred = await task
                if isinstance(pred, np.ndarray):
                    p = float(pred[0]) if (len(pred.shape) > 0 and pred.shape[0] > 0) else float(pred)
                else:
                    p = float(pred)
                p = max(0.0, min(1.0, p))
                out.append((name, p, self._calculate_model_confidence(p, name)))
            except Exception:
                continue  # dropped, weights renormalise over the rest (:175-181)
        return out

    @staticmethod
    def _calculate_model_confidence(p: float, name: str) -> float:
        return min(1.0, abs(p - 0.5) * 2 * _CONF_MULT.get(name, 0.5))

    def _combine(self, preds):
        if self.strategy == EnsembleStrategy.VOTING:
            votes = 0
            cs = 0.0
            for _, p, c in preds:
                if p > self.fraud_threshold:
                    votes += 1
                cs += c
            n = len(preds)
            return (votes / n if n > 0 else 0.0), (cs / n if n > 0 else 0.0)
        if self.strategy == EnsembleStrategy.STACKING:
            tc = sum(c for _, _, c in preds)
            if tc != 0:
                return sum(p * c for _, p, c in preds) / tc, tc / len(preds)
        tw = ws = cs = 0.0
        for name, p, c in preds:
            w = self.model_weights.get(name, 0.0)
            ws += p * w
            cs += c * w
            tw += w
        if tw == 0:
            return 0.5, 0.0
        return ws / tw, cs / tw

    def _make_decision(self, fp: float, conf: float) -> str:
        if conf < self.confidence_threshold:
            return "REVIEW"
        if fp >= 0.95:
            return "DECLINE"
        if fp >= 0.8:
            return "REVIEW"
        if fp >= 0.6:
            return "APPROVE_WITH_MONITORING"
        return "APPROVE"

    @staticmethod
    def _calculate_risk_level(fp: float) -> str:
        if fp >= 0.95:
            return "CRITICAL"
        if fp >= 0.8:
            return "HIGH"
        if fp >= 0.6:
            return "MEDIUM"
        if fp >= 0.3:
            return "LOW"
        return "VERY_LOW"

    def _generate_explanation(self, preds, features: Dict[str, Any]) -> Dict[str, Any]:
        total = sum(self.model_weights.get(n, 0) for n, _, _ in preds)
        contrib = {}
        for n, p, c in preds:
            w = self.model_weights.get(n, 0)
            contrib[n] = {"prediction": p, "weight": w, "contribution": (p * w / total) if total > 0 else 0,
                          "confidence": c}
        factors = []
        amount = features.get("amount", 0)
        if amount > 10000:
            factors.append(f"High transaction amount: ${amount:,.2f}")
        elif amount < 1:
            factors.append(f"Unusual low amount: ${amount:.2f}")
        hour = features.get("hour_of_day", 12)
        if hour < 6 or hour > 22:
            factors.append(f"Off-hours transaction: {hour}:00")
        pm = features.get("payment_method", "")
        if pm in ["crypto", "gift_card"]:
            factors.append(f"High-risk payment method: {pm}")
        importance = {}
        sub = features.get("features")
        if isinstance(sub, dict):
            imp = {k: min(abs(float(v)), 1.0) for k, v in sub.items() if isinstance(v, (int, float))}
            imp = {k: v for k, v in imp.items() if v > 0.1}
            importance = dict(sorted(imp.items(), key=lambda kv: kv[1], reverse=True)[:10])
        return {"model_contributions": contrib, "key_factors": factors, "feature_importance": importance}

    def _generate_cache_key(self, f: Dict[str, Any]) -> str:
        return "_".join(str(f.get(k, "")) for k in ("transaction_id", "amount", "user_id", "merchant_id",
                                                    "payment_method"))

    def _get_cached_prediction(self, key: str) -> Optional[Dict[str, Any]]:
        hit = self.prediction_cache.get(key)
        if hit is None:
            return None
        result, ts = hit
        if time.time() - ts < self.cache_ttl_seconds:
            return result
        del self.prediction_cache[key]
        return None

    def _cache_prediction(self, key: str, result: Dict[str, Any]) -> None:
        if len(self.prediction_cache) > 1000:
            oldest = min(self.prediction_cache, key=lambda k: self.prediction_cache[k][1])
            del self.prediction_cache[oldest]
        self.prediction_cache[key] = (result, time.time())

    # ------------------------------------------------------------------ micro-batch (GPU epilogue)
    def blend_params(self, names: List[str]) -> N.fd_blend_params:
        return FraudEngine.blend_params([self.model_weights.get(n, 0.0) for n in names],
                                        [_CONF_MULT.get(n, 0.5) for n in names], _STRATEGY_CODE[self.strategy],
                                        self.fraud_threshold, self.confidence_threshold)

    def score_matrix(self, X: np.ndarray) -> Dict[str, Any]:
        """Score prepared vectors (n, >=64). -> arrays: model probabilities per model, fraud_probability,
        confidence, decision / risk codes (fdengine._native.DECISIONS / RISK_LEVELS)."""
        mm = self.model_manager
        names = [n for n in self.config.get_enabled_models() if mm.is_model_loaded(n)]
        if not names:
            raise ValueError("No enabled models are loaded")
        n = X.shape[0]
        slots, ext, present = [], [], []
        for name in names:
            slot = mm.engine_slot(name)
            col = None
            ok = 1
            if slot < 0:  # host stand-in: one call for the whole batch, reference semantics
                try:
                    model = mm.models[name]
                    col = np.asarray(mm.predict_sync(name, model, self.config.get_model_config(name).model_type, X),
                                     dtype=np.float64).reshape(-1)
                    if col.shape[0] != n:
                        raise ValueError("stand-in returned the wrong number of rows")
                except Exception:
                    ok, col = 0, None
            elif slot == N.FD_SLOT_LSTM:
                ok, slot = 0, -1  # flat vectors carry no sequence: dropped, as the reference's LSTM is
            elif mm.models[name].kind == "xgboost" and X.shape[1] > mm.models[name].num_feature:
                ok = 0  # XGBoost rejects wider matrices; the reference drops the model
            elif mm.models[name].kind == "isolation_forest" and X.shape[1] != mm.models[name].num_feature:
                ok = 0  # sklearn's n_features_in_ check raises ValueError; the reference drops the model
            slots.append(slot)
            ext.append(col)
            present.append(ok)
        if not any(present):
            raise ValueError("No model predictions available")
        params = self.blend_params(names)
        mp, fp, conf, dec, risk = mm.engine.score_matrix(params, slots, X, ext, present)
        return {"models": names, "present": present, "model_probs": mp, "fraud_probability": fp, "confidence": conf,
                "decision": dec, "risk": risk}

    async def predict_batch(self, features_list: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
        t0 = time.time()
        if not features_list:
            return []
        # The reference scores each transaction's own vector: rows are grouped by their unpadded width (one
        # group in practice, 64), so a wide row only changes which models score THAT row.
        rows = [prepare_features(f)[0] for f in features_list]
        groups: Dict[int, List[int]] = {}
        for i, r in enumerate(rows):
            groups.setdefault(len(r), []).append(i)
        scored = {}
        for width, idx in groups.items():
            X = np.stack([rows[i] for i in idx])
            try:
                r = self.score_matrix(X)
            except ValueError:
                if len(groups) == 1:
                    raise
                r = None  # no model could score this width: those rows fail below, as predict() would
            for j, i in enumerate(idx):
                scored[i] = (r, j)
        per_txn_ms = (time.time() - t0) * 1000 / len(features_list)
        out = []
        for i, f in enumerate(features_list):
            r, j = scored[i]
            if r is None:
                raise ValueError("No model predictions available")
            preds = []
            for m, ok in enumerate(r["present"]):
                if not ok:
                    continue
                p = max(0.0, min(1.0, float(r["model_probs"][m, j])))
                preds.append((r["models"][m], p, self._calculate_model_confidence(p, r["models"][m])))
            fp = float(r["fraud_probability"][j])
            out.append({
                "fraud_probability": fp, "fraud_score": fp, "confidence": float(r["confidence"][j]),
                "risk_level": N.RISK_LEVELS[r["risk"][j]], "decision": N.DECISIONS[r["decision"][j]],
                "model_predictions": {n: p for n, p, _ in preds}, "model_confidences": {n: c for n, _, c in preds},
                "explanation": self._generate_explanation(preds, f) if self.enable_explanation else {},
                "ensemble_strategy": self.strategy.value, "processing_time_ms": per_txn_ms,
            })
        return out
