"""ORACLE — TEST INFRASTRUCTURE ONLY. Pure-Python restatement of
  FeatureProcessor.process_features  (services/ml-models/src/models/feature_processor.py:161-402)
  EnsemblePredictor._prepare_features (services/ml-models/src/models/ensemble_predictor.py:221-250)
pinned against the imported reference by tests/golden/feature_processor_cases.json.

Semantics restated (with the reference line each follows):
  * 41 definitions in declaration order (:66-147): value from the raw top-level dict, else the Flink
    `features` sub-dict, else default_value, else (required -> ValueError) the type default 0.0.
  * NUMERICAL (:227-240): float(v) (None -> 0.0), clamp with Python max/min against the bounds,
    then NaN/inf -> default_value (or 0.0). BINARY (:242-248): bool -> 1/0; str -> 1 if lower() in
    {'true','1','yes'}; else float(v) > 0.5. Conversion errors -> default_value or 0.0 (:273-275).
  * normalization is a no-op (scalers_fitted False, :159, :298).
  * derived (:330-373), appended in this order when present: amount_log (overwrites in place) and
    amount_sqrt if amount > 0; amount_to_user_avg_ratio if user_avg_amount > 0;
    amount_to_merchant_avg_ratio if merchant_avg_amount > 0; hourly_velocity_ratio if
    count_24h > 0; combined_device_ip_risk; is_business_hours; is_late_night; then string metadata.
  * _final_validation (:375-402) keeps finite numbers (non-finite -> default).
  * _prepare_features: numeric values in insertion order (bool counts: isinstance(True, int)),
    excluding metadata keys; zero-pad to 64; np.clip(-10, 10).
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

NUM, BIN = "numerical", "binary"
# (name, type, required, min, max, default) — feature_processor.py:66-147, in declaration order
DEFS: List[Tuple[str, str, bool, Optional[float], Optional[float], Optional[float]]] = [
    ("amount", NUM, True, 0.0, None, None),
    ("amount_log", NUM, False, None, None, 0.0),
    ("amount_percentile", NUM, False, 0.0, 100.0, None),
    ("amount_zscore", NUM, False, None, None, None),
    ("rounded_amount_frequency", NUM, False, 0.0, None, None),
    ("hour_of_day", NUM, False, 0, 23, 12),
    ("day_of_week", NUM, False, 0, 6, 1),
    ("is_weekend", BIN, False, None, None, 0),
    ("is_holiday", BIN, False, None, None, 0),
    ("time_since_last_transaction", NUM, False, 0.0, None, None),
    ("distance_from_home", NUM, False, 0.0, None, None),
    ("location_risk_score", NUM, False, 0.0, 1.0, None),
    ("country_risk_score", NUM, False, 0.0, 1.0, 0.5),
    ("timezone_mismatch", BIN, False, None, None, 0),
    ("user_transaction_count_1h", NUM, False, 0, None, None),
    ("user_transaction_count_24h", NUM, False, 0, None, None),
    ("user_total_amount_24h", NUM, False, 0.0, None, None),
    ("user_avg_amount", NUM, False, 0.0, None, None),
    ("user_unique_merchants_24h", NUM, False, 0, None, None),
    ("user_account_age_days", NUM, False, 0, None, None),
    ("merchant_transaction_count_1h", NUM, False, 0, None, None),
    ("merchant_fraud_rate", NUM, False, 0.0, 1.0, 0.0),
    ("merchant_avg_amount", NUM, False, 0.0, None, None),
    ("merchant_risk_score", NUM, False, 0.0, 1.0, 0.5),
    ("merchant_category_risk", NUM, False, 0.0, 1.0, 0.5),
    ("device_risk_score", NUM, False, 0.0, 1.0, 0.5),
    ("is_new_device", BIN, False, None, None, 0),
    ("ip_risk_score", NUM, False, 0.0, 1.0, 0.5),
    ("is_tor_ip", BIN, False, None, None, 0),
    ("is_vpn_ip", BIN, False, None, None, 0),
    ("velocity_score", NUM, False, 0.0, 1.0, 0.0),
    ("amount_velocity_1h", NUM, False, 0.0, None, None),
    ("transaction_velocity_5m", NUM, False, 0.0, None, None),
    ("payment_method_risk", NUM, False, 0.0, 1.0, 0.5),
    ("card_type_risk", NUM, False, 0.0, 1.0, 0.5),
    ("is_crypto_merchant", BIN, False, None, None, 0),
    ("is_gift_card_merchant", BIN, False, None, None, 0),
    ("cross_border_transaction", BIN, False, None, None, 0),
    ("payment_method_encoded", NUM, False, 0, 10, 0),
    ("merchant_category_encoded", NUM, False, 0, 20, 0),
    ("card_type_encoded", NUM, False, 0, 5, 0),
]
DEF_INDEX = {d[0]: i for i, d in enumerate(DEFS)}
METADATA = ("transaction_id", "user_id", "merchant_id", "timestamp", "currency", "payment_method")
EXCLUDED = {"transaction_id", "user_id", "merchant_id", "timestamp", "currency", "payment_method", "card_type"}
VECTOR_WIDTH = 64


def _fallback(default):
    return default if default is not None else 0.0


def validate(value: Any, ftype: str, lo, hi, default):
    try:
        if ftype == NUM:
            v = float(value) if value is not None else 0.0
            if lo is not None:
                v = max(v, lo)
            if hi is not None:
                v = min(v, hi)
            if math.isnan(v) or math.isinf(v):
                v = _fallback(default)
            return v
        if isinstance(value, bool):
            return 1.0 if value else 0.0
        if isinstance(value, str):
            return 1.0 if value.lower() in ("true", "1", "yes") else 0.0
        return 1.0 if float(value) > 0.5 else 0.0
    except (ValueError, TypeError):
        return _fallback(default)


def process_features(raw: Dict[str, Any]) -> Dict[str, Any]:
    flink = raw.get("features", {})
    out: Dict[str, Any] = {}
    for name, ftype, required, lo, hi, default in DEFS:
        if name in raw:
            value = raw[name]
        elif name in flink:
            value = flink[name]
        elif default is not None:
            value = default
        elif required:
            raise ValueError(f"Required feature '{name}' not found")
        else:
            value = 0.0
        out[name] = validate(value, ftype, lo, hi, default)
    # derived (:330-373)
    amount = out.get("amount", 0.0)
    if amount > 0:
        out["amount_log"] = np.log1p(amount)
        out["amount_sqrt"] = np.sqrt(amount)
    user_avg = out.get("user_avg_amount", 1.0)
    if user_avg > 0:
        out["amount_to_user_avg_ratio"] = amount / user_avg
    merchant_avg = out.get("merchant_avg_amount", 1.0)
    if merchant_avg > 0:
        out["amount_to_merchant_avg_ratio"] = amount / merchant_avg
    c1 = out.get("user_transaction_count_1h", 0)
    c24 = out.get("user_transaction_count_24h", 0)
    if c24 > 0:
        out["hourly_velocity_ratio"] = c1 / (c24 / 24)
    out["combined_device_ip_risk"] = (out.get("device_risk_score", 0.5) + out.get("ip_risk_score", 0.5)) / 2
    hour = out.get("hour_of_day", 12)
    out["is_business_hours"] = 1.0 if 9 <= hour <= 17 else 0.0
    out["is_late_night"] = 1.0 if hour < 6 or hour > 22 else 0.0
    for k, dflt in zip(METADATA, ("", "", "", "", "USD", "unknown")):
        out[k] = raw.get(k, dflt)
    # final validation (:375-402)
    for k, v in list(out.items()):
        if isinstance(v, (int, float)) and not np.isfinite(v):
            out[k] = _fallback(DEFS[DEF_INDEX[k]][5]) if k in DEF_INDEX else 0.0
    return out


def prepare_vector(processed: Dict[str, Any]) -> np.ndarray:
    vals = [float(v) for k, v in processed.items() if k not in EXCLUDED and isinstance(v, (int, float))]
    if "features" in processed and isinstance(processed["features"], dict):
        vals += [float(v) for v in processed["features"].values() if isinstance(v, (int, float))]
    while len(vals) < VECTOR_WIDTH:
        vals.append(0.0)
    return np.clip(np.array(vals).reshape(1, -1), -10, 10)


def numeric_keys(processed: Dict[str, Any]) -> List[str]:
    return [k for k, v in processed.items() if k not in EXCLUDED and isinstance(v, (int, float))]
