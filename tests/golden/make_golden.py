#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE's own Python
(AjayAlluri/realtime-fraud-detection @ /root/reference, services/ml-models/src) in the build
container. The reference never travels: only the input/output vectors written here do.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Reference code exercised (unchanged):
  models/feature_processor.py   FeatureProcessor.process_features            (:161-402)
  models/ensemble_predictor.py  EnsemblePredictor._prepare_features          (:221-250)
                                EnsemblePredictor.predict (blend, decision)  (:75-148, 252-369)
  models/model_manager.py       ModelManager.predict -> _predict_xgboost / _predict_sklearn /
                                _predict_tensorflow                          (:279-346)
Third-party modules the reference imports but this path does not execute are absent here and are
registered as empty modules so the import succeeds (ordinary ModuleNotFoundError otherwise):
xgboost (the XGBoost model is a deterministic stand-in object with predict_proba), tensorflow
(tf.keras.Model is only a type annotation). transformers, torch, sklearn are the installed ones.
The IsolationForest is a real sklearn 1.7.2 model trained with the reference trainer's recipe.

Outputs:
  feature_processor_cases.json  raw request dicts -> processed numeric key order + 64-wide vector
  ensemble_cases.json           raw request + stand-in probabilities -> reference predict() outputs, incl. the
                                processed request, the explanation dict and the prediction-cache key (a14)
  iforest_golden.npz            IF flattened arrays, inputs, sklearn apply/decision_function and the
                                reference _predict_sklearn probabilities
"""
import asyncio
import importlib.machinery
import json
import math
import sys
import types
from pathlib import Path

import numpy as np

sys.dont_write_bytecode = True
HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF_SRC = Path("/root/reference/services/ml-models/src")

sys.path.insert(0, str(REPO / "realtime-fraud-detection_amd"))


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m


def import_reference():
    _stub("xgboost", XGBClassifier=object)
    _stub("tensorflow", keras=types.SimpleNamespace(Model=object, models=types.SimpleNamespace()),
          config=types.SimpleNamespace())
    sys.path.insert(0, str(REF_SRC))
    from models.feature_processor import FeatureProcessor
    from models.ensemble_predictor import EnsemblePredictor
    from models.model_manager import ModelManager
    from utils.config import Config
    return FeatureProcessor, EnsemblePredictor, ModelManager, Config


# ------------------------------------------------------------------------------------ input cases

BRIDGED = ["amount_log", "hour_of_day", "day_of_week", "is_weekend", "merchant_fraud_rate", "is_new_device",
           "ip_risk_score", "user_avg_amount", "transaction_velocity_5m", "user_transaction_count_1h",
           "user_transaction_count_24h", "amount_velocity_1h", "user_total_amount_24h", "merchant_risk_score",
           "user_account_age_days", "merchant_avg_amount", "velocity_score", "user_unique_merchants_24h",
           "merchant_transaction_count_1h", "distance_from_home", "payment_method_encoded", "card_type_encoded",
           "merchant_category_encoded", "is_crypto_merchant", "cross_border_transaction"]
WEIRD = [float("nan"), float("inf"), -float("inf"), -5.0, 0.0, 1e9, "true", "yes", "no", "abc", "0.7", None, True,
         False, 3, -1, 25, 7, 0.5]


def raw_case(rng, i):
    amount = float(np.round(rng.lognormal(4, 1), 2))
    if i % 17 == 0:
        amount = 0.0
    if i % 23 == 0:
        amount = float(rng.choice([-3.5, 1e7, 12.0, 10.0]))
    c24 = int(rng.poisson(3))
    c1 = min(c24, int(rng.poisson(1)))
    feats = {
        "amount_log": math.log(amount + 1) if amount > -1 else 0.0,
        "hour_of_day": int(rng.integers(0, 24)),
        "day_of_week": int(rng.integers(1, 8)),
        "is_weekend": bool(rng.random() < 0.3),
        "merchant_fraud_rate": float(rng.choice([0.005, 0.01, 0.02, 0.08, 0.15, 0.05, 0.1])),
        "is_new_device": bool(rng.random() < 0.2),
        "ip_risk_score": float(rng.choice([0.1, 0.3])),
        "user_avg_amount": float(rng.lognormal(4, 1)) if rng.random() > 0.1 else 0.0,
        "transaction_velocity_5m": int(min(c1, rng.poisson(0.3))),
        "user_transaction_count_1h": c1,
        "user_transaction_count_24h": c24,
        "amount_velocity_1h": float(np.round(rng.lognormal(4, 1) * c1, 2)),
        "user_total_amount_24h": float(np.round(rng.lognormal(4, 1) * c24, 2)),
        "merchant_risk_score": float(rng.choice([0.2, 0.5, 0.8, 1.0])),
        "user_account_age_days": int(rng.integers(0, 730)),
        "merchant_avg_amount": float(rng.lognormal(4, 1)) if rng.random() > 0.1 else 0.0,
    }
    # perturb: drop keys, inject odd values and types, extra unknown keys
    for k in list(feats):
        r = rng.random()
        if r < 0.06:
            del feats[k]
        elif r < 0.10:
            feats[k] = WEIRD[int(rng.integers(0, len(WEIRD)))]
    if rng.random() < 0.3:
        feats["velocity_5min_count"] = int(rng.integers(0, 5))  # Flink-native name: ignored by FP
    raw = {"transaction_id": f"txn_{i:06d}", "user_id": f"user_{int(rng.integers(0, 500))}",
           "merchant_id": f"merchant_{int(rng.integers(0, 100))}", "amount": amount, "currency": "USD",
           "payment_method": str(rng.choice(["credit_card", "debit_card", "digital_wallet", "bank_transfer"])),
           "features": feats, "timestamp": "2025-09-05T12:00:00"}
    if rng.random() < 0.05:  # top-level override beats the features sub-dict
        raw["hour_of_day"] = int(rng.integers(0, 30))
    return raw


def jsonable(v):
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, (np.integer,)):
        return int(v)
    return v


def main():
    FeatureProcessor, EnsemblePredictor, ModelManager, Config = import_reference()
    from fdengine import synth
    from fdengine.forest import iforest_from_sklearn

    rng = np.random.default_rng(20250905)
    cfg = Config()
    fp = FeatureProcessor(cfg)

    # ---------------------------------------------------------------- FeatureProcessor + vector
    fp_cases = []
    for i in range(400):
        raw = raw_case(rng, i)
        try:
            processed = asyncio.run(fp.process_features(json.loads(json.dumps(raw))))
        except Exception as e:  # e.g. required feature missing
            fp_cases.append({"raw": raw, "error": type(e).__name__})
            continue
        vec = EnsemblePredictor._prepare_features(None, processed)
        keys = [k for k, v in processed.items()
                if k not in {"transaction_id", "user_id", "merchant_id", "timestamp", "currency", "payment_method",
                             "card_type"} and isinstance(v, (int, float))]
        fp_cases.append({"raw": raw, "numeric_keys": keys, "vector": [float(x) for x in vec[0]]})
    # the required-feature error path
    raw = raw_case(rng, 9999)
    del raw["amount"]
    try:
        asyncio.run(fp.process_features(raw))
        err = None
    except Exception as e:
        err = type(e).__name__
    fp_cases.append({"raw": raw, "error": err})
    (HERE / "feature_processor_cases.json").write_text(json.dumps(fp_cases, default=jsonable))

    # ---------------------------------------------------------------- IsolationForest (sklearn)
    Xtr = synth.feature_matrix(3000, 64, seed=4242).astype(np.float64)
    ifm = synth.isolation_forest(Xtr)
    fa = iforest_from_sklearn(ifm)
    Xif = np.array([c["vector"] for c in fp_cases if "vector" in c][:300], dtype=np.float64)
    Xif32 = Xif.astype(np.float32)
    apply = np.stack([e.apply(Xif32) for e in ifm.estimators_], 1).astype(np.int32)
    dfn = ifm.decision_function(Xif)

    class _Cfg:
        pass

    mm = ModelManager.__new__(ModelManager)  # only _predict_sklearn is used here
    ref_prob = np.array([asyncio.run(ModelManager._predict_sklearn(mm, ifm, Xif[i:i + 1]))[0]
                         for i in range(len(Xif))])
    np.savez_compressed(HERE / "iforest_golden.npz", offsets=fa.offsets, left=fa.left, right=fa.right,
                        feature=fa.feature, threshold=fa.threshold, default_left=fa.default_left,
                        leaf_value=fa.leaf_value, if_offset=fa.if_offset, if_denominator=fa.if_denominator,
                        num_feature=fa.num_feature, X=Xif, apply=apply, decision_function=dfn, ref_prob=ref_prob)

    # ---------------------------------------------------------------- EnsemblePredictor.predict
    class XgbStandIn:  # deterministic stand-in for xgb.XGBClassifier (predict_proba API)
        def __init__(self, p):
            self.p = p

        def predict_proba(self, X):
            return np.array([[1.0 - self.p, self.p]], dtype=np.float32)

    class LstmStandIn:  # keras-like: predict(X, verbose=0) -> (1, 2)
        def __init__(self, p, fail):
            self.p, self.fail = p, fail

        def predict(self, X, verbose=0):
            if self.fail:
                raise TypeError("stand-in failure (the reference's DummyModel also raises here)")
            return np.array([[1.0 - self.p, self.p]])

    ens_cases = []
    good = [c for c in fp_cases if "vector" in c]
    for strategy in ("weighted_average", "voting", "stacking"):
        cfg2 = Config()
        cfg2.disable_model("bert_text")
        cfg2.disable_model("graph_neural")
        cfg2.ensemble.strategy = strategy
        mm = ModelManager(cfg2)
        ep = EnsemblePredictor(mm, cfg2)
        for j in range(120):
            c = good[(j * 7 + len(strategy)) % len(good)]
            raw = json.loads(json.dumps(c["raw"]))
            raw["transaction_id"] = f"{strategy}_{j}"
            pick = rng.random()
            px = float(np.float32(rng.choice([rng.random(), 0.0, 1.0, 0.5, 0.97, 0.81, 0.61, 0.3])))
            pl = float(rng.random())
            lstm_fail = bool(rng.random() < 0.5)
            present = {"xgboost_primary": True, "lstm_sequential": True, "isolation_forest": True}
            mm.models = {}
            if pick > 0.1:
                mm.models["xgboost_primary"] = XgbStandIn(px)
            else:
                present["xgboost_primary"] = False
            mm.models["lstm_sequential"] = LstmStandIn(pl, lstm_fail)
            mm.models["isolation_forest"] = ifm
            processed = asyncio.run(fp.process_features(raw))
            out = asyncio.run(ep.predict(processed))
            ens_cases.append({
                "strategy": strategy, "raw": raw, "xgb_prob": px if present["xgboost_primary"] else None,
                "lstm_prob": None if lstm_fail else pl,
                "expected": {k: jsonable(out[k]) for k in ("fraud_probability", "confidence", "decision",
                                                            "risk_level")},
                "model_predictions": {k: float(v) for k, v in out["model_predictions"].items()},
                "model_confidences": {k: float(v) for k, v in out["model_confidences"].items()},
                "model_weights": {k: float(v) for k, v in ep.model_weights.items()},
                # a14: the explanation and the prediction-cache key the reference derives from this request
                "processed": processed,
                "explanation": out["explanation"],
                "cache_key": ep._generate_cache_key(processed),
            })
    (HERE / "ensemble_cases.json").write_text(json.dumps(ens_cases, default=jsonable))
    print(f"wrote {len(fp_cases)} feature cases, {len(ens_cases)} ensemble cases, IF golden {Xif.shape}")


if __name__ == "__main__":
    main()
