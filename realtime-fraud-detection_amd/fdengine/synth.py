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
                p_leaf: float = 0.0, base_score: float = 0.5, num_feature: Optional[int] = None,
                max_bin: Optional[int] = 256) -> dict:
    """Random gbtree trees in the XGBoost 2.0.3 JSON schema. p_leaf: chance a node at depth >= 2
    stops early (ragged trees exercise the perfect-tree padding). max_bin: split conditions are drawn
    from per-feature quantile cuts of X_ref, as XGBoost 2.0's default tree_method="hist" (max_bin=256)
    produces them (<= max_bin - 1 distinct thresholds per feature); None draws raw X_ref values."""
    rng = np.random.Generator(np.random.PCG64(seed))
    X_ref = np.asarray(X_ref, dtype=np.float32)
    cuts = {}
    if max_bin is not None:
        q = np.linspace(0.0, 1.0, max_bin + 1)[1:-1]
        for f in range(n_features):
            col = X_ref[:, f]
            col = col[~np.isnan(col)]
            cuts[f] = np.unique(np.quantile(col, q).astype(np.float32)) if len(col) else np.zeros(1, np.float32)
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
                if max_bin is not None:
                    thr = float(cuts[f][rng.integers(0, len(cuts[f]))])
                else:
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


# (category, risk level, avg amount, fraud rate): services/data-simulator/src/main/python/simulator.py:255-266
MERCHANT_CATEGORIES = (("retail", "low", 50.0, 0.01), ("grocery", "low", 25.0, 0.005),
                       ("gas_station", "medium", 40.0, 0.02), ("restaurant", "low", 35.0, 0.008),
                       ("online_retail", "medium", 75.0, 0.025), ("gambling", "high", 200.0, 0.15),
                       ("adult_entertainment", "high", 100.0, 0.12), ("pharmacy", "medium", 30.0, 0.01),
                       ("jewelry", "high", 500.0, 0.08), ("electronics", "medium", 300.0, 0.03))
# MerchantProfile.getRiskMultiplier() is referenced by FeatureExtractor.java:281 but the class is
# missing from the reference source; the engine takes the multiplier per merchant from the host and
# this is the build's declared table (clamped to [0,1] by FeatureProcessor as merchant_risk_score).
RISK_MULTIPLIER = {"low": 0.25, "medium": 0.5, "high": 0.9}


def _nonzero_u64(rng, n):
    k = rng.integers(1, np.iinfo(np.int64).max, size=n, dtype=np.int64).astype(np.uint64)
    return k | np.uint64(1) << np.uint64(63)


def population(n_users: int, n_merchants: int = 5000, seed: int = 42) -> dict:
    """Users (= cards) and merchants with the simulator's distributions (simulator.py:206-296).
    Card keys are random 64-bit values standing in for hash64(user_id)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    n_fp = rng.integers(1, 4, n_users)
    fps = _nonzero_u64(rng, n_users * 3).reshape(n_users, 3)
    fps[np.arange(3)[None, :] >= n_fp[:, None]] = 0
    cat = rng.integers(0, len(MERCHANT_CATEGORIES), n_merchants)
    return {
        "users": {
            "key": _nonzero_u64(rng, n_users),
            "avg_amount": rng.lognormal(4.0, 1.0, n_users),
            "account_age_days": rng.integers(0, 730, n_users).astype(np.int32),
            "device_fp": fps,
            "txn_frequency": (np.floor(rng.gamma(2.0, 2.0, n_users)) + 1).astype(np.int32),
        },
        "merchants": {
            "category": cat.astype(np.int32),
            "avg_amount": np.array([MERCHANT_CATEGORIES[c][2] for c in cat]) * rng.uniform(0.5, 2.0, n_merchants),
            "fraud_rate": np.array([MERCHANT_CATEGORIES[c][3] for c in cat]),
            "risk_multiplier": np.array([RISK_MULTIPLIER[MERCHANT_CATEGORIES[c][1]] for c in cat]),
        },
    }


def txn_stream(pop: dict, n: int, seed: int = 7, t0_ms: int = 1_757_030_400_000, rate_per_s: float = None,
               unknown_user_frac: float = 0.01, unknown_merchant_frac: float = 0.005) -> dict:
    """Transactions in arrival order (simulator.py:298-374): user/merchant uniform, amount =
    max(1, round(avg * N(1,.3) * N(1,.2), 2)) in integer cents, fraud patterns card_testing
    (U(1,5)) / account_takeover (new device) / synthetic (U(1000,5000)) with the simulator's
    probabilities (:107-127). Event time: Poisson arrivals at the population's aggregate rate
    (sum of txn_frequency / 86400 s unless rate_per_s is given) from t0_ms."""
    rng = np.random.Generator(np.random.PCG64(seed))
    U, M = pop["users"], pop["merchants"]
    nu, nm = len(U["key"]), len(M["category"])
    lam = rate_per_s if rate_per_s else max(float(U["txn_frequency"].sum()) / 86400.0, 1e-3)
    ts = t0_ms + np.floor(np.cumsum(rng.exponential(1000.0 / lam, n))).astype(np.int64)
    u = rng.integers(0, nu, n)
    key = U["key"][u].copy()
    unknown = rng.random(n) < unknown_user_frac
    key[unknown] = _nonzero_u64(rng, int(unknown.sum()))
    merchant = rng.integers(0, nm, n).astype(np.int32)
    merchant[rng.random(n) < unknown_merchant_frac] = -1
    base = U["avg_amount"][u] * rng.normal(1.0, 0.3, n) * rng.normal(1.0, 0.2, n)
    cents = np.maximum(100, np.rint(base * 100.0)).astype(np.int64)
    roll = rng.random(n)
    card_testing = roll < 0.02
    takeover = (roll >= 0.02) & (roll < 0.03)
    synthetic = (roll >= 0.03) & (roll < 0.035)
    cents[card_testing] = np.rint(rng.uniform(1.0, 5.0, int(card_testing.sum())) * 100).astype(np.int64)
    cents[synthetic] = np.rint(rng.uniform(1000.0, 5000.0, int(synthetic.sum())) * 100).astype(np.int64)
    fp_pick = rng.integers(0, 3, n)
    dfp = U["device_fp"][u, fp_pick]
    first = U["device_fp"][u, 0]
    dfp = np.where(dfp == 0, first, dfp)
    dfp[takeover] = _nonzero_u64(rng, int(takeover.sum()))
    ip_class = np.where(rng.random(n) < 0.05, 1, 2).astype(np.uint8)
    return {"card_key": key, "ts_ms": ts, "amount_cents": cents, "merchant": merchant, "device_fp": dfp,
            "ip_class": ip_class, "hour": np.full(n, 255, np.uint8), "weekend": np.full(n, 255, np.uint8),
            "is_fraud": roll < 0.055}


def isolation_forest(X_train: np.ndarray, n_estimators: int = 100, contamination: float = 0.05,
                     random_state: int = 42, max_samples="auto"):
    from sklearn.ensemble import IsolationForest
    m = IsolationForest(contamination=contamination, n_estimators=n_estimators, random_state=random_state,
                        max_samples=max_samples)
    m.fit(X_train)
    return m


# ------------------------------------------------------------------ hash-derived card populations
# For the sharded configurations (BASELINE config 4: 100M cards over 8 GPUs) every rank needs the
# attributes of the cards it owns and of the cards its own stream touches, without materialising the
# whole population: card i's attributes are a pure function of (i, seed).
_HM1 = np.uint64(0xff51afd7ed558ccd)
_HM2 = np.uint64(0xc4ceb9fe1a85ec53)


def _fmix64(k: np.ndarray) -> np.ndarray:
    k = np.asarray(k, np.uint64).copy()
    with np.errstate(over="ignore"):
        k ^= k >> np.uint64(33)
        k *= _HM1
        k ^= k >> np.uint64(33)
        k *= _HM2
        k ^= k >> np.uint64(33)
    return k


def _u01(ids: np.ndarray, seed: int, lane: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        h = _fmix64(np.asarray(ids, np.uint64) * np.uint64(0x9E3779B97F4A7C15)
                    + np.uint64((seed * 131 + lane) * 0x632BE59BD9B4E019 % (1 << 64)))
    return ((h >> np.uint64(11)).astype(np.float64) + 0.5) * (1.0 / (1 << 53))


def card_keys(ids, seed: int = 42) -> np.ndarray:
    """64-bit card key of card ids (stands in for hash64(user_id)); never 0."""
    ids = np.asarray(ids, np.int64).astype(np.uint64)
    with np.errstate(over="ignore"):
        return _fmix64(ids ^ np.uint64((seed * 0x2545F4914F6CDD1D) % (1 << 64))) | (np.uint64(1) << np.uint64(63))


def card_attrs(ids, seed: int = 42) -> dict:
    """Attributes of cards `ids` (int64 in [0, n_cards)) with the simulator's distributions
    (simulator.py:212-238: avg amount LogNormal(4,1), 1-3 device fingerprints, account age, transactions per day
    floor(Gamma(2, 2)) + 1 (:229), Gamma(2, 2) drawn as the sum of two Exp(2))."""
    from scipy.special import ndtri
    ids = np.asarray(ids, np.int64).astype(np.uint64)
    key = card_keys(ids, seed)
    n_fp = 1 + np.floor(_u01(ids, seed, 1) * 3).astype(np.int64)
    fps = np.stack([_fmix64(ids * np.uint64(4) + np.uint64(j + 1) + np.uint64(seed)) | (np.uint64(1) << np.uint64(63))
                    for j in range(3)], axis=1)
    fps[np.arange(3)[None, :] >= n_fp[:, None]] = 0
    freq = np.floor(-2.0 * np.log(_u01(ids, seed, 5)) - 2.0 * np.log(_u01(ids, seed, 6))) + 1.0
    return {"key": key, "avg_amount": np.exp(4.0 + ndtri(_u01(ids, seed, 2))),
            "account_age_days": np.floor(_u01(ids, seed, 3) * 730).astype(np.int32), "device_fp": fps,
            "txn_frequency": freq.astype(np.int16)}


def merchants_table(n_merchants: int = 5000, seed: int = 42) -> dict:
    return population(1, n_merchants, seed)["merchants"]


def owned_cards(n_cards: int, rank: int, world: int, seed: int = 42, chunk: int = 1 << 23) -> dict:
    """The cards GPU `rank` of `world` owns (fdengine.shard_of(key, world) == rank), with attributes."""
    from .engine import shard_of
    parts = []
    for a in range(0, n_cards, chunk):
        ids = np.arange(a, min(n_cards, a + chunk), dtype=np.int64)
        if world > 1:
            ids = ids[shard_of(card_keys(ids, seed), world) == rank]
        parts.append(card_attrs(ids, seed))
    return {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}


def txn_stream_cards(n_cards: int, merchants: dict, n: int, seed: int = 7, card_seed: int = 42,
                     t0_ms: int = 1_757_030_400_000, rate_per_s: float = 1000.0,
                     unknown_user_frac: float = 0.01, unknown_merchant_frac: float = 0.005) -> dict:
    """txn_stream over a hash-derived population of n_cards (same per-transaction distributions)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    u = rng.integers(0, n_cards, n)
    at = card_attrs(u, card_seed)
    pop = {"users": {"key": at["key"], "avg_amount": at["avg_amount"], "device_fp": at["device_fp"],
                     "txn_frequency": np.ones(n, np.int32)},
           "merchants": merchants}
    # draw the per-transaction fields with the user index being the identity over `at`
    tx = _txn_stream_indexed(pop, np.arange(n), rng, t0_ms, rate_per_s, unknown_user_frac, unknown_merchant_frac)
    tx["card_id"] = u  # population index of each transaction's card (unknown-user rows keep theirs)
    return tx


def _txn_stream_indexed(pop, u, rng, t0_ms, rate_per_s, unknown_user_frac, unknown_merchant_frac):
    U, M = pop["users"], pop["merchants"]
    n, nm = len(u), len(M["category"])
    ts = t0_ms + np.floor(np.cumsum(rng.exponential(1000.0 / rate_per_s, n))).astype(np.int64)
    key = U["key"][u].copy()
    unknown = rng.random(n) < unknown_user_frac
    key[unknown] = _nonzero_u64(rng, int(unknown.sum()))
    merchant = rng.integers(0, nm, n).astype(np.int32)
    merchant[rng.random(n) < unknown_merchant_frac] = -1
    base = U["avg_amount"][u] * rng.normal(1.0, 0.3, n) * rng.normal(1.0, 0.2, n)
    cents = np.maximum(100, np.rint(base * 100.0)).astype(np.int64)
    roll = rng.random(n)
    card_testing = roll < 0.02
    takeover = (roll >= 0.02) & (roll < 0.03)
    synthetic = (roll >= 0.03) & (roll < 0.035)
    cents[card_testing] = np.rint(rng.uniform(1.0, 5.0, int(card_testing.sum())) * 100).astype(np.int64)
    cents[synthetic] = np.rint(rng.uniform(1000.0, 5000.0, int(synthetic.sum())) * 100).astype(np.int64)
    fp_pick = rng.integers(0, 3, n)
    dfp = U["device_fp"][u, fp_pick]
    first = U["device_fp"][u, 0]
    dfp = np.where(dfp == 0, first, dfp)
    dfp[takeover] = _nonzero_u64(rng, int(takeover.sum()))
    ip_class = np.where(rng.random(n) < 0.05, 1, 2).astype(np.uint8)
    return {"card_key": key, "ts_ms": ts, "amount_cents": cents, "merchant": merchant, "device_fp": dfp,
            "ip_class": ip_class, "hour": np.full(n, 255, np.uint8), "weekend": np.full(n, 255, np.uint8),
            "is_fraud": roll < 0.055}


# ------------------------------------------------------------------ extended profiles + context (feature map)
# vocabularies (simulator.py:330-332 payment/type/card lists; kyc statuses :221-223; risk levels :255-266)
PAYMENT_METHODS = ("credit_card", "debit_card", "digital_wallet", "bank_transfer", "crypto", "prepaid_card",
                   "gift_card", "wire_transfer")
TXN_TYPES = ("purchase", "withdrawal", "transfer", "refund")
CARD_TYPES = ("visa", "mastercard", "amex", "discover")
KYC_STATUSES = ("verified", "pending", "rejected")
RISK_LEVELS = ("low", "medium", "high")


def vocab_flags():
    """-> (payment code -> isHighRiskPaymentMethod, type code -> is "refund"), 256 flags each."""
    pay = np.zeros(256, np.uint8)
    for i, p in enumerate(PAYMENT_METHODS):
        pay[i] = any(s in p.lower() for s in ("prepaid", "gift", "crypto", "wire"))
    ref = np.zeros(256, np.uint8)
    ref[TXN_TYPES.index("refund")] = 1
    return pay, ref


def users_ext(pop: dict, seed: int = 5, null_frac: float = 0.05) -> dict:
    """Extended UserProfile fields with the simulator's distributions (simulator.py:212-238) and some nulls."""
    rng = np.random.Generator(np.random.PCG64(seed))
    n = len(pop["users"]["key"])
    kyc = rng.choice(3, n, p=[0.85, 0.12, 0.03]).astype(np.uint8)
    d = {"key": pop["users"]["key"], "risk_score": rng.beta(2, 8, n), "kyc_status": kyc,
         "verified": (kyc == 0).astype(np.uint8), "pref_start": rng.integers(6, 11, n).astype(np.int8),
         "pref_end": rng.integers(18, 24, n).astype(np.int8), "weekend_activity": rng.uniform(0.3, 1.0, n),
         "online_preference": rng.uniform(0.5, 0.95, n), "intl_preference": rng.uniform(0.0, 0.1, n),
         "txn_frequency": pop["users"]["txn_frequency"].astype(np.int32),
         "has_patterns": (rng.random(n) < 0.9).astype(np.uint8)}
    for f in ("risk_score", "weekend_activity", "intl_preference"):
        d[f] = d[f].copy()
        d[f][rng.random(n) < null_frac] = np.nan
    d["weekend_activity"][rng.random(n) < 0.1] = 0.2  # exercise the < 0.3 rule
    d["pref_start"][rng.random(n) < null_frac] = -1
    d["kyc_status"][rng.random(n) < null_frac] = 255
    d["txn_frequency"][rng.random(n) < null_frac] = -1
    return d


def merchants_ext(pop: dict, seed: int = 6) -> dict:
    rng = np.random.Generator(np.random.PCG64(seed))
    M = pop["merchants"]
    n = len(M["category"])
    rl = np.array([RISK_LEVELS.index(MERCHANT_CATEGORIES[c][1]) for c in M["category"]], np.uint8)
    d = {"avg_amount": M["avg_amount"].copy(), "risk_level": rl, "blacklisted": (rng.random(n) < 0.02).astype(np.uint8),
         "category": M["category"].astype(np.uint8), "high_risk_category": (rl == 2).astype(np.uint8),
         "open_hour": rng.integers(6, 11, n).astype(np.uint8), "close_hour": rng.integers(20, 25, n).astype(np.uint8),
         "suspicious_name": (rng.random(n) < 0.05).astype(np.uint8)}
    d["avg_amount"][rng.random(n) < 0.05] = np.nan
    d["risk_level"][rng.random(n) < 0.03] = 255
    d["open_hour"][rng.random(n) < 0.03] = 255
    d["suspicious_name"][rng.random(n) < 0.03] = 255
    return d


def txn_context(tx: dict, seed: int = 8) -> dict:
    rng = np.random.Generator(np.random.PCG64(seed))
    n = len(tx["ts_ms"])
    lat = rng.uniform(-70, 70, n)
    lon = rng.uniform(-180, 180, n)
    lat[rng.random(n) < 0.05] = np.nan
    lon[rng.random(n) < 0.05] = np.nan
    near = rng.random(n) < 0.1  # the (|lat| < 10 and |lon| < 10) high-risk box
    lat[near], lon[near] = rng.uniform(-9, 9, int(near.sum())), rng.uniform(-9, 9, int(near.sum()))
    mlat = lat + rng.normal(0, 2, n)
    mlon = lon + rng.normal(0, 2, n)
    mlat[rng.random(n) < 0.1] = np.nan
    fs = rng.beta(2, 5, n)
    fs[rng.random(n) < 0.3] = np.nan
    pay = rng.integers(0, len(PAYMENT_METHODS), n).astype(np.uint8)
    pay[rng.random(n) < 0.02] = 255
    tt = rng.integers(0, len(TXN_TYPES), n).astype(np.uint8)
    tt[rng.random(n) < 0.02] = 255
    ct = rng.integers(0, len(CARD_TYPES), n).astype(np.uint8)
    ct[rng.random(n) < 0.02] = 255
    ua = (rng.random(n) < 0.05).astype(np.uint8)
    ua[rng.random(n) < 0.05] = 255
    return {"geo_lat": lat, "geo_lon": lon, "merchant_lat": mlat, "merchant_lon": mlon, "payment_method": pay,
            "transaction_type": tt, "card_type": ct, "user_agent_flag": ua, "fraud_score": fs}


def window_stream(n_batches: int, batch: int, n_cards: int, n_merchants: int, seed: int = 0,
                  t0_ms: int = 1_756_684_800_000, batch_span_ms: int = 20_000, jitter_ms: int = 15_000,
                  late_frac: float = 0.01, late_ms: int = 900_000, unknown_merchant_frac: float = 0.05,
                  hot_merchant_frac: float = 0.1):
    """Micro-batches for the Flink window aggregates (a5): card keys drawn with a skew (some cards
    repeat within 5 minutes), event times advancing ~batch_span_ms per batch with out-of-order jitter
    (within the 10 s watermark lag and beyond it) plus a few very late events; payment-method codes with
    nulls, isFraud flags, incoming fraud scores with nulls; one hot merchant (large tumbling segments)."""
    rng = np.random.default_rng(seed)
    keys = card_keys(np.arange(n_cards, dtype=np.int64), seed=seed + 11)
    out = []
    for b in range(n_batches):
        base = t0_ms + b * batch_span_ms
        idx = np.minimum((rng.pareto(1.2, batch) * n_cards / 20).astype(np.int64), n_cards - 1)
        ts = base + rng.integers(0, batch_span_ms, batch) - rng.integers(0, jitter_ms, batch)
        late = rng.random(batch) < late_frac
        ts = np.where(late, ts - rng.integers(late_ms // 2, late_ms, batch), ts)
        merchant = rng.integers(0, n_merchants, batch).astype(np.int32)
        merchant = np.where(rng.random(batch) < hot_merchant_frac, 0, merchant).astype(np.int32)
        merchant = np.where(rng.random(batch) < unknown_merchant_frac, -1, merchant).astype(np.int32)
        cents = np.where(rng.random(batch) < 0.05, rng.integers(100_000, 2_000_000, batch),
                         rng.integers(1, 50_000, batch)).astype(np.int64)
        pm = rng.integers(0, 6, batch).astype(np.uint8)
        pm = np.where(rng.random(batch) < 0.1, 255, pm).astype(np.uint8)
        fraud = (rng.random(batch) < 0.05).astype(np.uint8)
        score = rng.random(batch)
        score = np.where(rng.random(batch) < 0.2, np.nan, score)
        out.append(dict(key=keys[idx], ts_ms=ts.astype(np.int64), amount_cents=cents, merchant=merchant,
                        payment_method=pm, is_fraud=fraud, fraud_score=score))
    return out


# ------------------------------------------------------------------ Kafka JSON messages (ingest codec)
SIM_PAYMENT_METHODS = ("credit_card", "debit_card", "digital_wallet", "bank_transfer")   # simulator.py:331
SIM_TXN_TYPES = ("purchase", "refund", "authorization")                                   # simulator.py:330
SIM_CARD_TYPES = ("visa", "mastercard", "amex", "discover")                               # simulator.py:332
USER_AGENTS = (
    "Mozilla/5.0 (Windows NT 10.0; Win64; x64) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/120.0 Safari/537.36",
    "Mozilla/5.0 (Macintosh; Intel Mac OS X 10_15_7) AppleWebKit/605.1.15 (KHTML, like Gecko) Version/17.1 Safari/605.1.15",
    "Mozilla/5.0 (iPhone; CPU iPhone OS 17_0 like Mac OS X) AppleWebKit/605.1.15 Mobile/15E148",
    "Mozilla/5.0 (compatible; Googlebot/2.1; +http://www.google.com/bot.html)",
    "Opera/9.80 (X11; Linux x86_64) Presto/2.12.388 Version/12.16",
    "curl/8.4.0",
    "python-requests/2.31",
    "Mozilla/5.0 (X11; Linux x86_64; rv:121.0) Gecko/20100101 Firefox/121.0 crawler-test",
    "Mozilla/5.0 (Linux; Android 14; Pixel 8) AppleWebKit/537.36 Chrome/120.0 Mobile Safari/537.36 é中",
)


def _uuid(rng) -> str:
    import uuid
    return str(uuid.UUID(bytes=rng.bytes(16), version=4))


def sim_population(n_users: int, n_merchants: int, seed: int = 42) -> dict:
    """User / merchant id strings in the simulator's formats (simulator.py:215, 231, 272)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    users = [f"user_{_uuid(rng)[:8]}" for _ in range(n_users)]
    fps = [[_uuid(rng) for _ in range(int(rng.integers(1, 4)))] for _ in range(n_users)]
    merchants = [f"merchant_{_uuid(rng)[:8]}" for _ in range(n_merchants)]
    avg = rng.lognormal(4.0, 1.0, n_users)
    return {"user_ids": users, "device_fps": fps, "merchant_ids": merchants, "avg_amount": avg}


def json_messages(sp: dict, n: int, seed: int = 7, t0_us: int = 1_757_030_400_000_000, rate_per_s: float = 50.0):
    """n transaction messages exactly as the simulator produces them: json.dumps(asdict(Transaction),
    default=str) (simulator.py:186, 319-374) — uuid transaction ids, isoformat() timestamps (microseconds,
    omitted when zero), Faker-style lat/lon (geolocation floats; merchant_location Decimals -> strings),
    booleans, fraud_type null / string, fraud_score floats with full repr."""
    import datetime as dt
    import json
    from decimal import Decimal
    rng = np.random.Generator(np.random.PCG64(seed))
    t = t0_us + np.cumsum(rng.exponential(1e6 / rate_per_s, n)).astype(np.int64)
    t[::97] = (t[::97] // 1_000_000) * 1_000_000  # some whole seconds: isoformat drops the fraction
    out = []
    nu, nm = len(sp["user_ids"]), len(sp["merchant_ids"])
    for i in range(n):
        u = int(rng.integers(0, nu))
        m = int(rng.integers(0, nm))
        when = dt.datetime(1970, 1, 1) + dt.timedelta(microseconds=int(t[i]))
        amount = max(1.0, round(float(sp["avg_amount"][u] * rng.normal(1.0, 0.3) * rng.normal(1.0, 0.2)), 2))
        roll = rng.random()
        fraud = roll < 0.055
        if roll < 0.02:
            amount = round(float(rng.uniform(1.0, 5.0)), 2)
        elif 0.03 <= roll < 0.035:
            amount = round(float(rng.uniform(1000.0, 5000.0)), 2)
        ip = (f"192.168.{rng.integers(0, 256)}.{rng.integers(1, 255)}" if rng.random() < 0.05 else
              f"10.{rng.integers(0, 256)}.{rng.integers(0, 256)}.{rng.integers(1, 255)}" if rng.random() < 0.03 else
              f"{rng.integers(1, 224)}.{rng.integers(0, 256)}.{rng.integers(0, 256)}.{rng.integers(1, 255)}")
        fps = sp["device_fps"][u]
        fp = fps[int(rng.integers(0, len(fps)))] if roll >= 0.03 or roll < 0.02 else _uuid(rng)
        glat, glon = round(float(rng.uniform(-90, 90)), 6), round(float(rng.uniform(-180, 180)), 6)
        mloc = {"lat": Decimal(f"{rng.uniform(-90, 90):.6f}"), "lon": Decimal(f"{rng.uniform(-180, 180):.6f}")}
        txn = {
            "transaction_id": _uuid(rng),
            "user_id": sp["user_ids"][u],
            "merchant_id": sp["merchant_ids"][m] if rng.random() > 0.01 else f"merchant_{_uuid(rng)[:8]}",
            "amount": amount,
            "currency": "USD",
            "transaction_type": SIM_TXN_TYPES[int(rng.integers(0, 3))],
            "payment_method": SIM_PAYMENT_METHODS[int(rng.integers(0, 4))],
            "card_type": SIM_CARD_TYPES[int(rng.integers(0, 4))],
            "card_last_four": str(int(rng.integers(1000, 10000))),
            "timestamp": when.isoformat(),
            "ip_address": ip,
            "device_id": fps[0],
            "device_fingerprint": fp,
            "user_agent": USER_AGENTS[int(rng.integers(0, len(USER_AGENTS)))],
            "geolocation": {"lat": glat, "lon": glon},
            "merchant_location": mloc,
            "is_weekend": when.weekday() >= 5,
            "hour_of_day": when.hour,
            "is_fraud": bool(fraud),
            "fraud_type": ("card_testing" if roll < 0.02 else "velocity_fraud") if fraud else None,
            "fraud_score": float(rng.uniform(0.7, 0.95)) if fraud else float(rng.uniform(0.0, 0.3)),
            "processing_time_ms": int(rng.integers(50, 501)),
        }
        out.append(json.dumps(txn, default=str).encode("utf-8"))
    return out


def fixed_ids(prefix: str, idx: np.ndarray) -> np.ndarray:
    """Id strings `prefix` + 8 hex digits (the simulator's f"user_{uuid[:8]}" shape) as a fixed-width
    uint8 matrix [n, len(prefix) + 8] (vectorised; no Python strings)."""
    idx = np.asarray(idx, np.uint64)
    mixed = _fmix64(idx ^ np.uint64(0x5DEECE66D)) & np.uint64(0xFFFFFFFF)
    hexd = np.frombuffer(b"0123456789abcdef", np.uint8)
    out = np.empty((len(idx), len(prefix) + 8), np.uint8)
    out[:, :len(prefix)] = np.frombuffer(prefix.encode(), np.uint8)
    for k in range(8):
        out[:, len(prefix) + k] = hexd[((mixed >> np.uint64(28 - 4 * k)) & np.uint64(15)).astype(np.int64)]
    return out


def hash64_fixed(mat: np.ndarray) -> np.ndarray:
    """fd_hash64 (fmix64(FNV-1a-64)) of every row of a fixed-width uint8 matrix, vectorised."""
    h = np.full(mat.shape[0], 0xcbf29ce484222325, np.uint64)
    prime = np.uint64(0x100000001b3)
    with np.errstate(over="ignore"):
        for k in range(mat.shape[1]):
            h = (h ^ mat[:, k].astype(np.uint64)) * prime
    return _fmix64(h)


def json_messages_fast(n: int, n_users: int, merchant_ids, seed: int = 7, t0_ms: int = 1_757_030_400_000,
                       rate_per_s: float = 2000.0, user_prefix: str = "user_", fp_prefix: str = "fp-"):
    """Simulator-format messages (the key order, separators and value forms of json.dumps(asdict(Transaction),
    default=str)) at bench scale: users are fixed_ids(user_prefix, i) with device fingerprints
    fixed_ids(fp_prefix, 3 i + k); the values follow json_messages' distributions."""
    import datetime as dt
    rng = np.random.Generator(np.random.PCG64(seed))
    u = rng.integers(0, n_users, n)
    m = rng.integers(0, len(merchant_ids), n)
    ts_us = (t0_ms * 1000 + np.cumsum(rng.exponential(1e6 / rate_per_s, n))).astype(np.int64)
    uid = fixed_ids(user_prefix, u)
    fpk = rng.integers(0, 3, n)
    fid = fixed_ids(fp_prefix, u * 3 + fpk)
    base = _u01(u.astype(np.uint64), 42, 0)
    avg = np.exp(4.0 + 1.0 * np.sqrt(2) * _erfinv(2 * base - 1))
    amount = np.maximum(1.0, np.round(avg * rng.normal(1.0, 0.3, n) * rng.normal(1.0, 0.2, n), 2))
    roll = rng.random(n)
    amount = np.where(roll < 0.02, np.round(rng.uniform(1, 5, n), 2), amount)
    amount = np.where((roll >= 0.03) & (roll < 0.035), np.round(rng.uniform(1000, 5000, n), 2), amount)
    fraud = roll < 0.055
    score = np.where(fraud, rng.uniform(0.7, 0.95, n), rng.uniform(0.0, 0.3, n))
    tt, pm, ct = rng.integers(0, 3, n), rng.integers(0, 4, n), rng.integers(0, 4, n)
    glat, glon = np.round(rng.uniform(-90, 90, n), 6), np.round(rng.uniform(-180, 180, n), 6)
    mlat, mlon = rng.uniform(-90, 90, n), rng.uniform(-180, 180, n)
    ua = rng.integers(0, len(USER_AGENTS), n)
    ip = rng.integers(0, 256, (n, 4))
    priv = rng.random(n) < 0.05
    txid = rng.integers(0, 1 << 62, n)
    uas = [json_str(a) for a in USER_AGENTS]
    out = []
    epoch = dt.datetime(1970, 1, 1)
    for i in range(n):
        when = epoch + dt.timedelta(microseconds=int(ts_us[i]))
        ipstr = f"192.168.{ip[i, 2]}.{ip[i, 3]}" if priv[i] else f"{ip[i, 0] or 1}.{ip[i, 1]}.{ip[i, 2]}.{ip[i, 3]}"
        f = bool(fraud[i])
        fpstr = fid[i].tobytes().decode()
        out.append((
            f'{{"transaction_id": "{txid[i]:016x}-tx", "user_id": "{uid[i].tobytes().decode()}", '
            f'"merchant_id": "{merchant_ids[m[i]]}", "amount": {float(amount[i])!r}, "currency": "USD", '
            f'"transaction_type": "{SIM_TXN_TYPES[tt[i]]}", "payment_method": "{SIM_PAYMENT_METHODS[pm[i]]}", '
            f'"card_type": "{SIM_CARD_TYPES[ct[i]]}", "card_last_four": "{1000 + txid[i] % 9000}", '
            f'"timestamp": "{when.isoformat()}", "ip_address": "{ipstr}", "device_id": "{fpstr}", '
            f'"device_fingerprint": "{fpstr}", "user_agent": {uas[ua[i]]}, '
            f'"geolocation": {{"lat": {float(glat[i])!r}, "lon": {float(glon[i])!r}}}, '
            f'"merchant_location": {{"lat": "{mlat[i]:.6f}", "lon": "{mlon[i]:.6f}"}}, '
            f'"is_weekend": {"true" if when.weekday() >= 5 else "false"}, "hour_of_day": {when.hour}, '
            f'"is_fraud": {"true" if f else "false"}, '
            f'"fraud_type": {chr(34) + "card_testing" + chr(34) if f else "null"}, '
            f'"fraud_score": {float(score[i])!r}, "processing_time_ms": {50 + txid[i] % 451}}}').encode())
    return out


def json_str(s: str) -> str:
    import json
    return json.dumps(s)


def _erfinv(y):
    from scipy.special import erfinv
    return erfinv(y)
