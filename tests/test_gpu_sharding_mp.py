"""GPU, multi-process: the sharded step (fdengine/sharding.py ShardedScorer + EngineShardBackend) with TWO real
ranks, each a process driving its own engine (its cards' state, windows and sink) on the one GPU of the test
box, exchanging over gloo (device tensors staged through the host; RCCL does the same exchanges on a
multi-GPU node). Checked against ONE unsharded engine that sees each step's two ingest batches concatenated in
rank order (the global arrival order):

* scores (fraud probability, confidence, decision, risk) bit-identical;
* Flink window aggregates (a5): the union of the ranks' user windows and every rank's merged merchant windows
  equal the unsharded engine's, field for field (one watermark via the all-reduce MAX; merchant partials
  merged by fd_merchant_windows_merge);
* sink aggregates (f3): hourly / daily / merchant-hour queries summed over ranks equal the unsharded ones.

The native step (fd_sharded_step over the engine's own communicators) needs RCCL, which refuses two ranks on one
device: its multi-rank test runs the ranks as threads over an in-process loopback of the RCCL API
(tests/test_gpu_sharding_loopback.py).
"""
import os
import pickle
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORLD, N_USERS, N_MERCH, B, STEPS = 2, 3000, 80, 4000, 3
MF = ("merchant", "window_start", "window_end", "first_ts", "last_ts", "count", "fraud_count", "high_risk_count",
      "unique_users", "unique_payment_methods", "total_amount", "fraud_amount", "avg_amount", "fraud_rate",
      "amount_stddev", "risk_score")
UF = ("user_key", "window_start", "window_end", "first_ts", "last_ts", "count", "fraud_count", "high_risk_count",
      "unique_merchants", "unique_payment_methods", "total_amount", "avg_amount", "fraud_rate", "velocity_score")


def _setup():
    from fdengine import iforest_from_sklearn, synth, xgboost_from_json_doc
    pop = synth.population(N_USERS, N_MERCH, seed=71)
    streams = [synth.txn_stream(pop, B * STEPS, seed=72 + r, rate_per_s=2.0) for r in range(WORLD)]
    pms = []
    for r in range(WORLD):
        rng = np.random.default_rng(80 + r)
        pm = rng.integers(0, 6, B * STEPS).astype(np.uint8)
        pm[rng.random(B * STEPS) < 0.1] = 255
        pms.append(pm)
    X = synth.feature_matrix(3000, 64, seed=73)
    xgb = xgboost_from_json_doc(synth.xgboost_doc(80, 8, 64, X, seed=74, p_leaf=0.1))
    ifm = iforest_from_sklearn(synth.isolation_forest(X.astype(np.float64), n_estimators=30))
    return pop, streams, pms, xgb, ifm


def _engine(pop, owned, xgb, ifm):
    from fdengine import FraudEngine
    U, M = pop["users"], pop["merchants"]
    e = FraudEngine(0)
    e.state_init(4 * N_USERS + 4096, 1, 16)
    e.load_users(U["key"][owned], U["avg_amount"][owned], U["account_age_days"][owned], U["device_fp"][owned])
    e.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    e.load_forest(0, xgb)
    e.load_forest(1, ifm)
    e.windows_init(1 << 16)
    e.sink_init(1 << 14, 1 << 16)
    return e


def _queries(sc, hours):
    days = sorted({h // 24 for h in hours})
    mids = np.repeat(np.arange(N_MERCH), len(hours))
    return {"hourly": sc.sink_query(1, hours), "daily": sc.sink_query(2, days),
            "merchant": sc.sink_query(3, np.tile(hours, N_MERCH), mids)}


def _hours(streams):
    return sorted({int(t) // 3_600_000 for s in streams for t in s["ts_ms"]})


def _run(sc, batches, n):
    """drive a ShardedScorer over prepared (txns, extras) device batches; -> scores, user windows, merchant windows"""
    scores, users, merchants = [], [], []
    for s, (part, extras) in enumerate(batches):
        out = sc.step(part, n, extras=extras, windows=True, sink=True, flush=s == len(batches) - 1)
        scores.append(np.stack([out[0].cpu().numpy(), out[1].cpu().numpy(), out[2].cpu().numpy().astype(np.float64),
                                out[3].cpu().numpy().astype(np.float64)]))
        uw, mw = sc.last_windows
        users.append(uw)
        merchants.append(mw)
    return np.concatenate(scores, axis=1), np.concatenate(users), np.concatenate(merchants)


def _dev_batch(tx, pm, sl):
    import torch

    from fdengine._native import TXN_FIELDS
    part = {f: torch.from_numpy(np.ascontiguousarray(tx[f][sl])).cuda() for f in TXN_FIELDS}
    extras = {"payment_method": torch.from_numpy(pm[sl].copy()).cuda(),
              "is_fraud": torch.from_numpy(tx["is_fraud"][sl].astype(np.uint8)).cuda()}
    return part, extras


def _worker(rank, port, outdir):
    import torch
    import torch.distributed as dist

    from fdengine import FraudEngine
    from fdengine.sharding import EngineShardBackend, ShardedScorer, owned_mask
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    eng = None
    try:
        torch.cuda.set_device(0)
        pop, streams, pms, xgb, ifm = _setup()
        eng = _engine(pop, owned_mask(pop["users"]["key"], rank, WORLD), xgb, ifm)
        params = FraudEngine.blend_params([0.4 / 0.45, 0.05 / 0.45], [1.0, 0.5])
        sc = ShardedScorer(EngineShardBackend(eng, params, [0, 1]), rank, WORLD)
        batches = [_dev_batch(streams[rank], pms[rank], slice(s * B, (s + 1) * B)) for s in range(STEPS)]
        scores, users, merchants = _run(sc, batches, B)
        torch.cuda.synchronize()
        with open(os.path.join(outdir, f"rank{rank}.pkl"), "wb") as f:
            pickle.dump({"scores": scores, "users": users, "merchants": merchants,
                         "sink": _queries(sc, _hours(streams)), "counts": sc.last_counts}, f)
    finally:
        if eng is not None:
            eng.close()
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rows(recs, fields, key):
    return sorted((tuple(r[f].item() for f in fields) for r in recs), key=lambda t: tuple(t[i] for i in key))


@pytest.mark.timeout(300)
def test_two_ranks_on_one_gpu_match_unsharded_engine(tmp_path):
    import torch
    import torch.multiprocessing as mp

    from fdengine import FraudEngine
    from fdengine.sharding import EngineShardBackend, ShardedScorer
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    got = [pickle.load(open(tmp_path / f"rank{r}.pkl", "rb")) for r in range(WORLD)]
    assert all(min(g["counts"][1]) > 0 for g in got)  # both owners received transactions

    pop, streams, pms, xgb, ifm = _setup()
    ref = _engine(pop, np.ones(N_USERS, bool), xgb, ifm)
    try:
        params = FraudEngine.blend_params([0.4 / 0.45, 0.05 / 0.45], [1.0, 0.5])
        sc = ShardedScorer(EngineShardBackend(ref, params, [0, 1]), 0, 1)
        cat = {k: np.concatenate([np.concatenate([streams[r][k][s * B:(s + 1) * B] for r in range(WORLD)])
                                  for s in range(STEPS)]) for k in streams[0]}
        pm = np.concatenate([np.concatenate([pms[r][s * B:(s + 1) * B] for r in range(WORLD)]) for s in range(STEPS)])
        n = WORLD * B
        batches = [_dev_batch(cat, pm, slice(s * n, (s + 1) * n)) for s in range(STEPS)]
        scores, users, merchants = _run(sc, batches, n)
        torch.cuda.synchronize()
        q = _queries(sc, _hours(streams))
    finally:
        ref.close()
    assert len(users) > 100 and len(merchants) > 50  # windows fired
    for r in range(WORLD):  # rank r's ingest rows are the r-th B-slice of every step's concatenated batch
        exp = np.concatenate([scores[:, s * n + r * B:s * n + (r + 1) * B] for s in range(STEPS)], axis=1)
        np.testing.assert_array_equal(got[r]["scores"], exp)
    got_users = np.concatenate([g["users"] for g in got])
    assert _rows(got_users, UF, (1, 0)) == _rows(users, UF, (1, 0))
    for r in range(WORLD):
        assert _rows(got[r]["merchants"], MF, (1, 0)) == _rows(merchants, MF, (1, 0))
        for k in ("hourly", "daily", "merchant"):
            np.testing.assert_array_equal(got[r]["sink"][k], q[k])


def _stream_worker(rank, port, outdir):
    import torch
    import torch.distributed as dist

    from fdengine import FraudEngine
    from fdengine.sharding import EngineShardBackend, ShardedScorer, owned_mask
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    eng = None
    try:
        torch.cuda.set_device(0)
        pop, streams, pms, xgb, ifm = _setup()
        eng = _engine(pop, owned_mask(pop["users"]["key"], rank, WORLD), xgb, ifm)
        params = FraudEngine.blend_params([0.4 / 0.45, 0.05 / 0.45], [1.0, 0.5])
        sc = ShardedScorer(EngineShardBackend(eng, params, [0, 1], pipelined=True), rank, WORLD, native=False)
        assert sc.streaming and not sc.native
        parts = [_dev_batch(streams[rank], pms[rank], slice(s * B, (s + 1) * B))[0] for s in range(STEPS)]
        outs = []
        for s in range(STEPS):
            pre = (parts[s + 1], B) if s + 1 < STEPS else None
            out = sc.step(parts[s], B, prefetch=pre)
            host = [torch.empty(o.shape, dtype=o.dtype, pin_memory=True) for o in out]
            for h, o in zip(host, out):
                h.copy_(o, non_blocking=True)
            outs.append(host)  # the device outputs are dropped at once (allocator reuse under the streams)
        torch.cuda.synchronize()
        scores = np.concatenate([np.stack([h[0].numpy(), h[1].numpy(), h[2].numpy().astype(np.float64),
                                           h[3].numpy().astype(np.float64)]) for h in outs], axis=1)
        with open(os.path.join(outdir, f"srank{rank}.pkl"), "wb") as f:
            pickle.dump({"scores": scores, "counts": sc.last_counts}, f)
    finally:
        if eng is not None:
            eng.close()
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_ranks_streaming_step_matches_oracle(tmp_path):
    """The streaming sharded step (partition + count exchange of the next batch launched one step ahead on a
    forward stream, records landing behind an event, fd_score_records_pipelined, results back on a second process
    group) with two real ranks on the one GPU, against the CPU oracle chain over the global arrival order
    (step-major, then ingest rank, then index): fraud probability, confidence, decision, risk bit-identical."""
    import torch.multiprocessing as mp
    mp.spawn(_stream_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    _check_against_oracle([pickle.load(open(tmp_path / f"srank{r}.pkl", "rb")) for r in range(WORLD)])


def _check_against_oracle(got):
    import oracle
    from oracle.features_c import OracleFeatureState
    assert all(min(g["counts"][1]) > 0 for g in got)
    pop, streams, _, xgb, ifm = _setup()
    U, M = pop["users"], pop["merchants"]
    st = OracleFeatureState(4 * N_USERS + 4096, 1, 16)
    st.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    st.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    exp = [[] for _ in range(WORLD)]
    for s in range(STEPS):
        for r in range(WORLD):
            part = {k: v[s * B:(s + 1) * B] for k, v in streams[r].items()}
            _, V = st.run(part, want_raw=False)
            px, _, _ = oracle.xgb_predict(xgb, V)
            pi, _, _ = oracle.iforest_predict(ifm, V)
            fp, conf, dec, risk = oracle.blend_weighted(np.stack([px.astype(np.float64), pi]),
                                                        [0.4 / 0.45, 0.05 / 0.45], [1.0, 0.5])
            exp[r].append(np.stack([fp, conf, dec.astype(np.float64), risk.astype(np.float64)]))
    for r in range(WORLD):
        g, e = got[r]["scores"], np.concatenate(exp[r], axis=1)
        # probabilities within the north-star 1e-5 (the f32 XGBoost sigmoid may differ by an ulp from the oracle's);
        # decision / risk exact except where the oracle's value sits within 1e-6 of a threshold
        assert np.abs(g[0] - e[0]).max() <= 1e-5 and np.abs(g[1] - e[1]).max() <= 1e-5
        near = np.zeros(g.shape[1], bool)
        for thr in (0.3, 0.6, 0.8, 0.95):
            near |= np.abs(e[0] - thr) < 1e-6
        near |= np.abs(e[1] - 0.7) < 1e-6
        assert ((g[2] == e[2]) | near).all() and ((g[3] == e[3]) | near).all()
        assert (g[2] == e[2]).mean() > 0.999
