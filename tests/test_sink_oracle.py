"""CPU: known answers of the RedisTransactionSink aggregate restatement (oracle/sink_ref.py;
RedisTransactionSink.java:140-262)."""
from oracle.sink_ref import SinkOracle, java_div

H = 3_600_000


def test_java_division_truncates():
    assert java_div(7, 2) == 3 and java_div(-7, 2) == -3 and java_div(-1, H) == 0


def test_hourly_daily_merchant_known_answers():
    o = SinkOracle()
    t0 = 1_757_030_400_000  # 2025-09-05T00:00:00Z, an hour and day boundary
    o.process(11, 10.0, t0 + 5, 3, False, 0.9)
    o.process(11, 2.5, t0 + H - 1, 3, True, None)
    o.process(12, 1.25, t0 + H, 3, False, 0.7)      # next hour; 0.7 is not > 0.7
    o.process(13, 4.0, t0 + 2 * H, None, True, 0.71)  # merchantId null: no merchant aggregation
    h0, h1, h2 = t0 // H, t0 // H + 1, t0 // H + 2
    a = o.redis[f"hourly:{h0}"]
    assert (a["total_count"], a["total_amount"], a["fraud_count"], a["high_risk_count"]) == (2, 12.5, 1, 1)
    assert a["fraud_rate"] == 0.5 and a["avg_amount"] == 6.25
    assert o.redis[f"hourly:{h1}"]["high_risk_count"] == 0
    assert o.redis[f"hourly:{h2}"]["high_risk_count"] == 1
    d = o.redis[f"daily:{t0 // 86_400_000}"]
    assert (d["total_count"], d["fraud_count"]) == (4, 2) and d["total_amount"] == 17.75
    m = o.redis[f"merchant:3:{h0}"]
    assert m["unique_user_count"] == 1 and m["total_count"] == 2
    assert f"merchant:None:{h2}" not in o.redis and not any(k.endswith(f":{h2}") and k.startswith("merchant")
                                                             for k in o.redis)
