"""TEST INFRASTRUCTURE ONLY (oracle) — never imported by the product path (fdengine/).

Line-by-line restatement of RedisTransactionSink.updateAggregations and its three helpers
(services/flink-jobs/src/main/java/com/frauddetection/sinks/RedisTransactionSink.java:140-262) with a dict standing
in for Redis (RedisService.storeAggregation / getAggregation, RedisService.java:246-276):

  hourKey = timestamp / 3_600_000, dayKey = timestamp / 86_400_000   (Java long division: truncation)  :142-144
  hourly:{hour}   total_count += 1; total_amount += amount (double, arrival order); fraud_count += isFraud;
                  high_risk_count += fraudScore > 0.7; fraud_rate = fraud / count; avg = amount / count   :165-194
  daily:{day}     the same without high_risk_count                                                    :199-222
  merchant:{id}:{hour}  + unique_users set, unique_user_count; skipped when merchantId is null          :227-262

`last_updated` (System.currentTimeMillis) is wall-clock and not restated. The Redis TTL (1800 s, processing
time) is not applied: the engine's retention is explicit. Parity vs Java unpinned (no JDK);
the restatement is pinned by the known-answer tests in tests/test_sink_oracle.py.
"""
from __future__ import annotations


def java_div(a: int, b: int) -> int:
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


class SinkOracle:
    def __init__(self):
        self.redis = {}

    def _get(self, key):
        return self.redis.get(key, {})

    def process(self, user_key: int, amount: float, ts_ms: int, merchant, is_fraud: bool, fraud_score):
        hour = java_div(ts_ms, 3_600_000)
        day = java_div(ts_ms, 86_400_000)
        self._hourly(amount, is_fraud, fraud_score, hour)
        self._daily(amount, is_fraud, day)
        self._merchant(user_key, amount, is_fraud, merchant, hour)

    def _hourly(self, amount, is_fraud, fraud_score, hour):
        key = f"hourly:{hour}"
        cur = self._get(key)
        total_count = cur.get("total_count", 0) + 1
        total_amount = cur.get("total_amount", 0.0) + (amount if amount is not None else 0.0)
        fraud_count = cur.get("fraud_count", 0) + (1 if is_fraud is True else 0)
        high = cur.get("high_risk_count", 0) + (1 if (fraud_score is not None and fraud_score == fraud_score
                                                        and fraud_score > 0.7) else 0)
        self.redis[key] = {"total_count": total_count, "total_amount": total_amount, "fraud_count": fraud_count,
                           "high_risk_count": high, "fraud_rate": fraud_count / total_count,
                           "avg_amount": total_amount / total_count}

    def _daily(self, amount, is_fraud, day):
        key = f"daily:{day}"
        cur = self._get(key)
        total_count = cur.get("total_count", 0) + 1
        total_amount = cur.get("total_amount", 0.0) + (amount if amount is not None else 0.0)
        fraud_count = cur.get("fraud_count", 0) + (1 if is_fraud is True else 0)
        self.redis[key] = {"total_count": total_count, "total_amount": total_amount, "fraud_count": fraud_count,
                           "fraud_rate": fraud_count / total_count, "avg_amount": total_amount / total_count}

    def _merchant(self, user_key, amount, is_fraud, merchant, hour):
        if merchant is None:
            return
        key = f"merchant:{merchant}:{hour}"
        cur = self._get(key)
        total_count = cur.get("total_count", 0) + 1
        total_amount = cur.get("total_amount", 0.0) + (amount if amount is not None else 0.0)
        fraud_count = cur.get("fraud_count", 0) + (1 if is_fraud is True else 0)
        users = set(cur.get("unique_users", ()))
        users.add(user_key)
        self.redis[key] = {"merchant_id": merchant, "total_count": total_count, "total_amount": total_amount,
                           "fraud_count": fraud_count, "fraud_rate": fraud_count / total_count,
                           "avg_amount": total_amount / total_count, "unique_users": users,
                           "unique_user_count": len(users)}

    def run_batch(self, b: dict):
        """b: window_stream-style batch (key, ts_ms, amount_cents, merchant (-1 = null), is_fraud, fraud_score)."""
        for i in range(len(b["key"])):
            m = int(b["merchant"][i])
            fs = float(b["fraud_score"][i]) if "fraud_score" in b else None
            self.process(int(b["key"][i]) or 1, int(b["amount_cents"][i]) / 100.0, int(b["ts_ms"][i]),
                         None if m < 0 else m, bool(b["is_fraud"][i]) if "is_fraud" in b else False,
                         None if fs is None or fs != fs else fs)
