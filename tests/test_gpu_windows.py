"""GPU parity of the Flink window aggregates (row a5): fd_windows_step_* (windows.hip: device event logs,
rocPRIM radix sort, segmented reduction) vs oracle/windows_ref.py on the same seeded micro-batch
streams — out-of-order and very late events, unknown merchants, null payment methods / scores, a hot
merchant, empty batches, end-of-input flush. Bar: every field bit-exact (counts and times are integers;
amounts exact cents / 100; scores and std-dev the same f64 operations). Parity vs Java/Flink unpinned."""
import math

import numpy as np
import pytest

from fdengine import synth
from oracle import windows_ref as W

pytestmark = pytest.mark.gpu

UF = ("user_key", "window_start", "window_end", "first_ts", "last_ts", "count", "fraud_count",
      "high_risk_count", "unique_merchants", "unique_payment_methods", "total_amount", "avg_amount",
      "fraud_rate", "velocity_score")
MF = ("merchant", "window_start", "window_end", "first_ts", "last_ts", "count", "fraud_count",
      "high_risk_count", "unique_users", "unique_payment_methods", "total_amount", "fraud_amount",
      "avg_amount", "fraud_rate", "amount_stddev", "risk_score")


def _oracle_batch(b):
    return [dict(key=int(b["key"][i]), ts=int(b["ts_ms"][i]), cents=int(b["amount_cents"][i]),
                 merchant=int(b["merchant"][i]), pm=int(b["payment_method"][i]), fraud=bool(b["is_fraud"][i]),
                 score=float(b["fraud_score"][i])) for i in range(len(b["key"]))]


def _rows(recs, fields, sort_by):
    rows = [tuple((r[f].item() if hasattr(r[f], "item") else r[f]) for f in fields) for r in recs]
    return sorted(rows, key=lambda t: tuple(t[i] for i in sort_by))


def _compare(gpu, orc, fields, sort_by):
    g = _rows(gpu, fields, sort_by)
    o = _rows(orc, fields, sort_by)
    assert len(g) == len(o)
    for a, b in zip(g, o):
        for f, x, y in zip(fields, a, b):
            if isinstance(y, float):
                assert x == y or (math.isnan(x) and math.isnan(y)), (f, a, b)
            else:
                assert x == y, (f, a, b)


def _run(engine, batches, device=False, log_capacity=1 << 16):
    import torch
    engine.state_init(1 << 15, 0, 4)
    engine.windows_init(log_capacity)
    orc = W.WindowOracle()
    nu = nm = 0
    for bi, b in enumerate(batches + [None]):
        flush = b is None
        if flush:
            b = {k: v[:0] for k, v in batches[0].items()}
        if device:
            t = {k: torch.from_numpy(np.ascontiguousarray(v)).to("cuda") for k, v in b.items()}
            txn = dict(card_key=t["key"].data_ptr(), ts_ms=t["ts_ms"].data_ptr(),
                       amount_cents=t["amount_cents"].data_ptr(), merchant=t["merchant"].data_ptr())
            ins = {k: t[k].data_ptr() for k in ("payment_method", "is_fraud", "fraud_score")}
            gu, gm = engine.windows_step_device(txn, len(b["key"]), ins, flush=flush)
        else:
            gu, gm = engine.windows_step_host(b["key"], b["ts_ms"], b["amount_cents"], b["merchant"],
                                              b["payment_method"], b["is_fraud"], b["fraud_score"], flush=flush)
        ou, om = orc.step(_oracle_batch(b), flush=flush)
        _compare(gu, ou, UF, (0, 1))
        _compare(gm, om, MF, (0, 1))
        assert engine.windows_stats()["watermark"] == (orc.wm if orc.wm is not None else -(1 << 63))
        nu += len(gu)
        nm += len(gm)
    return nu, nm


@pytest.mark.parametrize("device", [False, True])
def test_windows_stream_parity(engine, device):
    batches = synth.window_stream(12, 3000, 400, 60, seed=5)
    nu, nm = _run(engine, batches, device=device)
    assert nu > 1000 and nm > 50


def test_windows_hot_key_and_empty_batches(engine):
    # few cards and one merchant: long segments in both sorts; empty batches in between
    batches = synth.window_stream(8, 2000, 5, 2, seed=9, hot_merchant_frac=0.8, batch_span_ms=200_000)
    empty = {k: v[:0] for k, v in batches[0].items()}
    batches = [batches[0], empty] + batches[1:4] + [empty, empty] + batches[4:]
    _run(engine, batches)


def test_windows_big_time_jump_and_late(engine):
    # a batch hours ahead fires every open window at once; the next batch is entirely late
    a = synth.window_stream(3, 1000, 50, 10, seed=2)
    b = synth.window_stream(2, 1000, 50, 10, seed=3, t0_ms=1_756_684_800_000 + 5 * 3_600_000)
    c = synth.window_stream(1, 500, 50, 10, seed=4)
    _run(engine, a + b + c)


def test_windows_errors(engine):
    from fdengine._native import NativeError
    engine.state_init(1 << 12, 0, 4)
    engine.windows_init(1000)
    b = synth.window_stream(1, 1001, 10, 5, seed=1)[0]
    with pytest.raises(NativeError, match="log full"):
        engine.windows_step_host(b["key"], b["ts_ms"], b["amount_cents"], b["merchant"])
    b = synth.window_stream(2, 500, 400, 5, seed=1)
    engine.windows_step_host(b[0]["key"], b[0]["ts_ms"], b[0]["amount_cents"], b[0]["merchant"])
    with pytest.raises(NativeError, match="result capacity"):
        engine.windows_step_host(b[1]["key"], b[1]["ts_ms"], b[1]["amount_cents"], b[1]["merchant"],
                                 flush=True, user_cap=1)
