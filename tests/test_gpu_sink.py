"""GPU parity of the RedisTransactionSink bucket aggregates ((f) rank 3; sink.hip) vs oracle/sink_ref.py on
seeded micro-batch streams: hourly / daily / merchant-hour keys, isFraud, fraudScore > 0.7, null merchants, hot
merchants and cards, eviction. Bars: counts, fraud / high-risk counts and distinct users bit-exact; fraud_rate
bit-exact (the same f64 division of exact integers); amounts within 1e-9 relative (exact cents / 100 vs the
reference's sequential double sum) and avg within 1e-5 absolute. Parity vs Java unpinned."""
import numpy as np
import pytest

from fdengine import synth
from fdengine._native import FD_AGG_DAILY, FD_AGG_HOURLY, FD_AGG_MERCHANT
from oracle.sink_ref import SinkOracle

pytestmark = pytest.mark.gpu


def _keys(o):
    hourly, daily, merch = [], [], []
    for k in o.redis:
        p = k.split(":")
        if p[0] == "hourly":
            hourly.append(int(p[1]))
        elif p[0] == "daily":
            daily.append(int(p[1]))
        else:
            merch.append((int(p[1]), int(p[2])))
    return sorted(hourly), sorted(daily), sorted(merch)


def _check(engine, o):
    hourly, daily, merch = _keys(o)
    for kind, keys, name in ((FD_AGG_HOURLY, hourly, "hourly"), (FD_AGG_DAILY, daily, "daily")):
        got = engine.sink_query(kind, keys)
        assert got["found"].all()
        for g, k in zip(got, keys):
            e = o.redis[f"{name}:{k}"]
            assert g["total_count"] == e["total_count"] and g["fraud_count"] == e["fraud_count"]
            if name == "hourly":
                assert g["high_risk_count"] == e["high_risk_count"]
            assert g["fraud_rate"] == e["fraud_rate"]
            assert abs(g["total_amount"] - e["total_amount"]) <= 1e-9 * max(1.0, abs(e["total_amount"]))
            assert abs(g["avg_amount"] - e["avg_amount"]) <= 1e-5
    m = np.array([k[0] for k in merch], np.int32)
    h = np.array([k[1] for k in merch], np.int64)
    got = engine.sink_query(FD_AGG_MERCHANT, h, m)
    assert got["found"].all()
    for g, (mm, hh) in zip(got, merch):
        e = o.redis[f"merchant:{mm}:{hh}"]
        assert (g["total_count"], g["fraud_count"], g["unique_user_count"]) == \
               (e["total_count"], e["fraud_count"], e["unique_user_count"])
        assert abs(g["total_amount"] - e["total_amount"]) <= 1e-9 * max(1.0, abs(e["total_amount"]))
    # absent keys are reported as not found
    assert not engine.sink_query(FD_AGG_HOURLY, [hourly[0] - 1000])["found"].any()
    return len(hourly), len(daily), len(merch)


@pytest.mark.parametrize("device", [False, True])
def test_sink_stream_parity(engine, device):
    import torch
    batches = synth.window_stream(10, 4000, 300, 40, seed=7, batch_span_ms=900_000)
    engine.sink_init(1 << 14, 1 << 16)
    o = SinkOracle()
    for b in batches:
        if device:
            t = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in b.items()}
            engine.sink_update_device({"card_key": t["key"].data_ptr(), "ts_ms": t["ts_ms"].data_ptr(),
                                       "amount_cents": t["amount_cents"].data_ptr(),
                                       "merchant": t["merchant"].data_ptr()}, len(b["key"]),
                                      {"is_fraud": t["is_fraud"].data_ptr(), "fraud_score": t["fraud_score"].data_ptr()})
        else:
            engine.sink_update_host(b["key"], b["ts_ms"], b["amount_cents"], b["merchant"], b["is_fraud"],
                                    b["fraud_score"])
        o.run_batch(b)
    nh, nd, nm = _check(engine, o)
    assert nh >= 3 and nd >= 1 and nm > 100


def test_sink_eviction(engine):
    batches = synth.window_stream(8, 3000, 200, 30, seed=9, batch_span_ms=1_800_000)
    engine.sink_init(1 << 13, 1 << 15)
    o = SinkOracle()
    for b in batches:
        engine.sink_update_host(b["key"], b["ts_ms"], b["amount_cents"], b["merchant"], b["is_fraud"],
                                b["fraud_score"])
        o.run_batch(b)
    hourly, _, merch = _keys(o)
    cut = hourly[len(hourly) // 2]
    kept_e, kept_u = engine.sink_evict_before(cut)
    old = [k for k in hourly if k < cut]
    new = [k for k in hourly if k >= cut]
    assert not engine.sink_query(FD_AGG_HOURLY, old)["found"].any()
    got = engine.sink_query(FD_AGG_HOURLY, new)
    assert got["found"].all()
    assert [int(x) for x in got["total_count"]] == [o.redis[f"hourly:{k}"]["total_count"] for k in new]
    keep_m = [(m, h) for m, h in merch if h >= cut]
    keep_d = [d for d in _keys(o)[1] if d * 24 + 23 >= cut]  # a day is kept while any of its hours is
    assert kept_e == len(new) + len(keep_m) + len(keep_d)
    assert kept_u == sum(o.redis[f"merchant:{m}:{h}"]["unique_user_count"] for m, h in keep_m)
    # updates after eviction keep counting the kept buckets exactly
    last = batches[-1]
    engine.sink_update_host(last["key"], last["ts_ms"], last["amount_cents"], last["merchant"], last["is_fraud"],
                            last["fraud_score"])
    o.run_batch(last)
    got = engine.sink_query(FD_AGG_HOURLY, new)
    assert [int(x) for x in got["total_count"]] == [o.redis[f"hourly:{k}"]["total_count"] for k in new]


def test_sink_capacity_error(engine):
    from fdengine._native import NativeError
    b = synth.window_stream(1, 2000, 500, 400, seed=3, batch_span_ms=40 * 3_600_000)[0]
    engine.sink_init(16, 1 << 12)
    with pytest.raises(NativeError, match="aggregate table full"):
        engine.sink_update_host(b["key"], b["ts_ms"], b["amount_cents"], b["merchant"])
