"""ORACLE — TEST INFRASTRUCTURE ONLY. Pure-Python restatement of the Java feature half of the path
for small cases, sequential in arrival order (the reference is per-element):

  FeatureExtractor.extractAllFeatures   fl/features/FeatureExtractor.java:50-87 (the extractors used
                                        by the bridged features, :92-363, null-profile branches
                                        :243-251 / :287-295)
  velocity read  RedisService.getVelocityMetrics  fl/services/RedisService.java:198-207
  velocity write RedisTransactionSink.updateVelocityWindow fl/sinks/RedisTransactionSink.java:116-135
                 (count += 1, amount += amt; key TTL 3600 s refreshed on every write, RedisService:47,188)
  (fl/ = services/flink-jobs/src/main/java/com/frauddetection/)

then the Flink -> FeatureProcessor name bridge (the reference's names do not match,
fact 8) and the pinned FeatureProcessor + _prepare_features restatement (features_ref.py).

Declared engine semantics (PARITY UNPINNED: no JDK, no reference tests):
  * per card (the reference's user_id, hashed to a u64 key) the extractor READS velocity, then the
    sink WRITES it (read-before-write), transactions of a card in arrival order;
  * window_mode 0 "redis_compat": one session counter per card; a read at t sees the previous write
    at t0 iff t - t0 <= 3,600,000 ms (Redis expires a key when now > expire_at); the 5min / 1hour /
    24hour "windows" are identical (fact 6); sums are kept as integer cents (exact);
  * window_mode 1 "sliding": true windows over the card's last K events, W in {300, 3600, 86400} s,
    counting prior events e with t - W < e.ts <= t;
  * unknown user (no profile): FeatureExtractor's null branch (no user_avg_amount, age 0, device
    unknown); unknown merchant: fraud rate 0.1, risk multiplier 2.0;
  * merchant fraud rate null -> 0.05 (:264-265); risk multiplier per merchant supplied by the host.
"""
from __future__ import annotations

import math
from typing import Dict, List

import numpy as np

from . import features_ref as FR

TTL_MS = 3_600_000
WINDOWS_MS = (300_000, 3_600_000, 86_400_000)

# raw (bridged Flink) feature columns produced per transaction, in this order
RAW_COLUMNS = ("amount", "amount_log_java", "hour", "day_of_week", "is_weekend", "merchant_fraud_rate",
               "is_new_device", "ip_risk_score", "user_avg_amount", "velocity_5min_count",
               "velocity_1hour_count", "velocity_24hour_count", "velocity_1hour_amount",
               "velocity_24hour_amount", "merchant_risk_multiplier", "account_age_days")


def utc_hour_dow(ts_ms: int):
    days = ts_ms // 86_400_000
    hour = (ts_ms - days * 86_400_000) // 3_600_000
    dow = (days + 3) % 7 + 1  # ISO: 1970-01-01 was a Thursday (4)
    return int(hour), int(dow)


class CardState:
    __slots__ = ("cnt", "sum_cents", "last_ts", "ring")

    def __init__(self):
        self.cnt, self.sum_cents, self.last_ts, self.ring = 0, 0, None, []


class FeatureState:
    def __init__(self, window_mode: int = 0, ring_k: int = 16):
        self.mode, self.K = window_mode, ring_k
        self.cards: Dict[int, CardState] = {}
        self.users: Dict[int, dict] = {}
        self.merchants: List[dict] = []

    def load_users(self, keys, avg_amount, account_age, device_fp):
        for i, k in enumerate(keys):
            self.users[int(k)] = {"avg": float(avg_amount[i]), "age": int(account_age[i]),
                                  "fps": {int(x) for x in device_fp[i] if int(x) != 0}}

    def load_merchants(self, fraud_rate, risk_mult):
        self.merchants = [{"fr": float(f), "mult": float(m)} for f, m in zip(fraud_rate, risk_mult)]

    # ---------------------------------------------------------------- one transaction
    def step(self, key, ts, cents, merchant, device_fp, ip_class, hour_in, weekend_in):
        key, ts, cents = int(key), int(ts), int(cents)
        amount = cents / 100.0
        hour, dow = utc_hour_dow(ts)
        if hour_in != 255:
            hour = int(hour_in)
        weekend = (dow >= 6) if weekend_in == 255 else bool(weekend_in)
        u = self.users.get(key)
        if 0 <= merchant < len(self.merchants):
            m = self.merchants[merchant]
            mfr = 0.05 if math.isnan(m["fr"]) else m["fr"]
            mult = m["mult"]
        else:
            mfr, mult = 0.1, 2.0
        known = u is not None and device_fp != 0 and int(device_fp) in u["fps"]
        ip = float("nan") if ip_class == 0 else (0.1 if ip_class == 1 else 0.3)
        if u is None:
            avg, age = float("nan"), 0
        else:
            avg = 0.0 if math.isnan(u["avg"]) else u["avg"]
            age = u["age"]
        st = self.cards.setdefault(key, CardState())
        # velocity READ (extractor), then WRITE (sink)
        if self.mode == 0:
            live = st.last_ts is not None and ts - st.last_ts <= TTL_MS
            c, s = (st.cnt, st.sum_cents) if live else (0, 0)
            counts, sums = (c, c, c), (s, s, s)
            st.cnt, st.sum_cents, st.last_ts = c + 1, s + cents, ts
        else:
            counts, sums = [], []
            for W in WINDOWS_MS:
                ev = [e for e in st.ring if ts - W < e[0] <= ts]
                counts.append(len(ev))
                sums.append(sum(e[1] for e in ev))
            st.ring.append((ts, cents))
            if len(st.ring) > self.K:
                st.ring.pop(0)
        return (amount, math.log(amount + 1) if amount > -1 else (float("-inf") if amount == -1 else float("nan")),
                hour, dow, 1.0 if weekend else 0.0, mfr, 0.0 if known else 1.0, ip, avg,
                counts[0], counts[1], counts[2], sums[1] / 100.0, sums[2] / 100.0, mult, age)

    def run(self, txns: dict):
        n = len(txns["card_key"])
        raw = np.zeros((n, len(RAW_COLUMNS)), np.float64)
        for i in range(n):
            raw[i] = self.step(txns["card_key"][i], txns["ts_ms"][i], txns["amount_cents"][i], txns["merchant"][i],
                               txns["device_fp"][i], txns["ip_class"][i], txns["hour"][i], txns["weekend"][i])
        return raw


def bridged_dict(raw_row) -> dict:
    """Flink feature names -> FeatureProcessor names (the build's declared bridge)."""
    r = list(raw_row)
    d = {"amount_log": r[1], "hour_of_day": int(r[2]), "day_of_week": int(r[3]), "is_weekend": bool(r[4]),
         "merchant_fraud_rate": r[5], "is_new_device": bool(r[6]),
         "transaction_velocity_5m": int(r[9]), "user_transaction_count_1h": int(r[10]),
         "user_transaction_count_24h": int(r[11]), "amount_velocity_1h": r[12], "user_total_amount_24h": r[13],
         "merchant_risk_score": r[14], "user_account_age_days": int(r[15])}
    if not math.isnan(r[7]):
        d["ip_risk_score"] = r[7]
    if not math.isnan(r[8]):
        d["user_avg_amount"] = r[8]
    return d


def vectors(raw: np.ndarray, txn_ids=None) -> np.ndarray:
    """raw bridged values -> the reference scoring vectors (n, 64) f64 via the pinned restatement."""
    out = np.zeros((len(raw), FR.VECTOR_WIDTH), np.float64)
    for i, r in enumerate(raw):
        req = {"transaction_id": f"t{i}", "user_id": "u", "merchant_id": "m", "amount": float(r[0]),
               "currency": "USD", "payment_method": "credit_card", "features": bridged_dict(r),
               "timestamp": ""}
        out[i] = FR.prepare_vector(FR.process_features(req))[0]
    return out
