"""Known-answer tests of the window-aggregate oracle (oracle/windows_ref.py, row a5) — hand-computed
windows for WindowProcessor's user-velocity (sliding 5 min / 1 min) and merchant (tumbling 1 h)
aggregates under micro-batch watermarks. Parity vs Java/Flink unpinned (no JDK / Flink, no reference
fixtures); these pin the restatement's semantics: assignment, firing, lateness, scores."""
import math

import numpy as np

from oracle import windows_ref as W

T0 = 1_756_684_800_000  # 2025-09-01T00:00:00Z, a multiple of 1 h


def ev(key, ts, cents, merchant=0, pm=255, fraud=False, score=float("nan")):
    return dict(key=key, ts=ts, cents=cents, merchant=merchant, pm=pm, fraud=fraud, score=score)


def test_sliding_assignment_and_firing():
    o = W.WindowOracle()
    # one event at T0 + 90 s: in the windows starting T0-180 s .. T0+60 s (5 windows)
    u, m = o.step([ev(7, T0 + 90_000, 1234, merchant=3)])
    assert (u, m) == ([], [])                        # watermark T0+79_999: nothing ends yet
    assert o.wm == T0 + 90_000 - 10_000 - 1
    u, m = o.step([ev(8, T0 + 130_000, 1)])          # watermark T0+119_999: [T0-180s, T0+120s) fires
    assert [(r["user_key"], r["window_start"], r["window_end"]) for r in u] == [(7, T0 - 180_000, T0 + 120_000)]
    r = u[0]
    assert (r["count"], r["first_ts"], r["last_ts"], r["unique_merchants"]) == (1, T0 + 90_000, T0 + 90_000, 1)
    assert r["total_amount"] == 12.34 and r["avg_amount"] == 12.34
    assert m == []
    u, m = o.step([], flush=True)                    # end of input: everything fires
    assert sorted((r["user_key"], r["window_start"]) for r in u) == sorted(
        [(7, T0 + s) for s in (-120_000, -60_000, 0, 60_000)] + [(8, T0 + s) for s in range(-120_000, 180_000, 60_000)])
    assert [(r["merchant"], r["window_start"], r["count"]) for r in m] == [(3, T0, 1), (0, T0, 1)]


def test_late_event_dropped_after_fire():
    o = W.WindowOracle()
    o.step([ev(1, T0 + 10_000, 100)])
    u, _ = o.step([ev(2, T0 + 200_000, 100)])        # watermark T0+189_999 fires ends <= T0+190_000
    fired = {(r["user_key"], r["window_start"]) for r in u}
    assert (1, T0 - 240_000) in fired and (1, T0 - 120_000) in fired
    # a late event for card 1 at T0+5 s: its windows ending <= watermark are gone; the ones still open take it
    u, _ = o.step([ev(1, T0 + 5_000, 50)])
    assert u == []
    u, _ = o.step([], flush=True)
    c1 = {r["window_start"]: r for r in u if r["user_key"] == 1}
    assert set(c1) == {T0 - 60_000, T0}               # the windows still open at the late arrival
    assert all(r["count"] == 2 and r["total_amount"] == 1.5 for r in c1.values())
    assert all(r["first_ts"] == T0 + 5_000 and r["last_ts"] == T0 + 10_000 for r in c1.values())


def test_velocity_score_and_counts():
    o = W.WindowOracle()
    evs = [ev(5, T0 + 1000 * i, 60_000, merchant=9 if i < 20 else 10, pm=i % 3, fraud=i < 3,
              score=0.9 if i % 2 else float("nan")) for i in range(22)]
    o.step(evs)
    u, _ = o.step([], flush=True)
    r = next(r for r in u if r["window_start"] == T0)
    assert r["count"] == 22 and r["fraud_count"] == 3 and r["high_risk_count"] == 11
    assert r["unique_merchants"] == 2 and r["unique_payment_methods"] == 3
    assert r["total_amount"] == 13200.0
    # 22 > 20: +0.4; 13200 > 10000: +0.3; fraud 3/22*0.4; diversity 2/22 < 0.2: +0.2 -> min(1, ...)
    assert r["velocity_score"] == min(1.0, 0.4 + 0.3 + (3 / 22) * 0.4 + 0.2)
    s = W.velocity_score(6, 100_001, 0, 6)           # 6 > 5: 0.1; 1000.01 > 1000: 0.1; div 1.0
    assert s == 0.1 + 0.1


def test_merchant_aggregate_and_stddev():
    o = W.WindowOracle()
    cents = [100, 250, 99_999, 100, 100_000]
    evs = [ev(k, T0 + 60_000 * i, c, merchant=4, fraud=(i == 2)) for i, (k, c) in enumerate(zip([1, 2, 1, 1, 3], cents))]
    evs.append(ev(9, T0 + 1, 777, merchant=-1))      # unknown merchant: not aggregated by merchant
    o.step(evs)
    _, m = o.step([], flush=True)
    assert len(m) == 1
    r = m[0]
    assert (r["merchant"], r["count"], r["unique_users"], r["fraud_count"]) == (4, 5, 3, 1)
    assert r["fraud_amount"] == 999.99 and r["total_amount"] == sum(cents) / 100
    sd = W.exact_stddev(cents)
    assert math.isclose(sd, W.java_stddev([c / 100 for c in cents]), rel_tol=1e-14)
    assert r["amount_stddev"] == sd
    # 1/5*0.5; stddev/avg = 0.93.. < 2; diversity 3/5
    assert r["risk_score"] == 0.1


def test_stddev_exact_vs_twopass_random():
    rng = np.random.default_rng(3)
    for n in (2, 3, 17, 1000):
        c = [int(x) for x in rng.integers(1, 2_000_000, n)]
        assert math.isclose(W.exact_stddev(c), W.java_stddev([x / 100 for x in c]), rel_tol=1e-12)


def test_empty_and_no_advance():
    o = W.WindowOracle()
    assert o.step([]) == ([], [])
    assert o.step([], flush=True) == ([], [])
    o.step([ev(1, T0, 1)])
    wm = o.wm
    assert o.step([ev(1, T0 - 50_000, 1)]) == ([], [])   # older batch max: watermark does not regress
    assert o.wm == wm
