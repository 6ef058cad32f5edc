"""CPU: card-hash sharding — the shard function, the stable partition, and the
ShardedScorer exchange protocol at world_size 2 over gloo, against one unsharded oracle run.

The per-rank compute is an oracle-backed backend (features + forests + blend restated on the CPU);
on the GPU the same ShardedScorer drives libfdengine.so (tests/test_gpu_sharding.py). Parity bar:
every rank's results equal the unsharded oracle's for the same transactions bit for bit, i.e. the
exchange preserves each card's arrival order and returns every result to its transaction."""
import os
import socket

import numpy as np
import pytest

from oracle import route_ref as R


def test_shard_function_matches_library():
    from fdengine.engine import shard_of
    rng = np.random.default_rng(5)
    keys = rng.integers(0, 2**63, 50000, dtype=np.int64).astype(np.uint64)
    keys[:4] = [0, 1, 2**64 - 1, 2**63]
    for G in (1, 2, 3, 4, 7, 8, 64):
        a, b = shard_of(keys, G), R.shard_of(keys, G)
        np.testing.assert_array_equal(a, b)
        assert a.min() >= 0 and a.max() < G
    c = np.bincount(R.shard_of(keys, 8), minlength=8)
    assert c.min() > 0.95 * len(keys) / 8  # balanced


def test_shard_bits_independent_of_table_slot_bits():
    """owner uses the high half of fmix64, the card table's home slot the low bits: owned keys must
    still cover every residue of the owner's table mask."""
    keys = np.arange(1, 200001, dtype=np.uint64)
    own = R.shard_of(keys, 8) == 3
    slots = R.fmix64(keys[own]) & np.uint64(1023)
    assert len(np.unique(slots)) == 1024


def test_partition_is_stable_and_complete():
    from fdengine import synth
    pop = synth.population(500, 50, seed=2)
    tx = synth.txn_stream(pop, 3000, seed=3, rate_per_s=5.0)
    rec, counts = R.partition(tx, 4)
    assert counts.sum() == 3000
    own = R.shard_of(rec["key"], 4)
    assert (np.diff(own) >= 0).all()  # owner-major
    for s in range(4):
        seq = rec["seq"][own == s].astype(np.int64)
        assert (np.diff(seq) > 0).all()  # arrival order kept inside each owner group
    assert sorted(rec["seq"].tolist()) == list(range(3000))
    back = R.records_to_txns(rec)
    for f in ("card_key", "ts_ms", "amount_cents", "merchant", "device_fp"):
        np.testing.assert_array_equal(back[f], np.asarray(tx[f])[rec["seq"].astype(np.int64)])


# ------------------------------------------------------------------ world_size-2 gloo run
N_USERS, N_MERCH, B, STEPS, WORLD = 400, 60, 700, 4, 2


def _models():
    import fdengine
    from fdengine import synth
    X = synth.feature_matrix(2000, 64, seed=31)
    xgb = fdengine.xgboost_from_json_doc(synth.xgboost_doc(40, 6, 64, X, seed=32, p_leaf=0.1))
    ifm = fdengine.iforest_from_sklearn(synth.isolation_forest(X.astype(np.float64), n_estimators=15))
    return xgb, ifm


def _streams():
    from fdengine import synth
    pop = synth.population(N_USERS, N_MERCH, seed=21)
    # each rank ingests its own stream over the SAME card population
    return pop, [synth.txn_stream(pop, B * STEPS, seed=40 + r, rate_per_s=3.0) for r in range(WORLD)]


WEIGHTS = [0.4 / 0.45, 0.05 / 0.45]
MULTS = [1.0, 0.5]


class OracleShardBackend:
    """Test-side backend: the per-rank compute of the sharded step restated on the CPU."""

    def __init__(self, rank, world, pop, xgb, ifm):
        import torch
        from oracle.features_c import OracleFeatureState
        self.torch, self.xgb, self.ifm = torch, xgb, ifm
        U, M = pop["users"], pop["merchants"]
        own = R.shard_of(U["key"], world) == rank
        self.state = OracleFeatureState(4096, 1, 8)
        self.state.load_users(U["key"][own], U["avg_amount"][own], U["account_age_days"][own], U["device_fp"][own])
        self.state.load_merchants(M["fraud_rate"], M["risk_multiplier"])
        self.scored = 0

    def partition(self, txns, n, G):
        rec, counts = R.partition({k: v.numpy() for k, v in txns.items()}, G)
        t = self.torch
        return t.from_numpy(rec.view(np.uint8).reshape(n, 48).copy()), t.from_numpy(counts)

    def score_records(self, rec, m):
        import oracle
        res = np.zeros(m, R.RESULT)
        if m:
            r = rec.numpy().reshape(-1).view(R.RECORD)
            _, V = self.state.run(R.records_to_txns(r), want_raw=False)
            px, _, _ = oracle.xgb_predict(self.xgb, V)
            pi, _, _ = oracle.iforest_predict(self.ifm, V)
            fp, conf, dec, risk = oracle.blend_weighted(np.stack([px.astype(np.float64), pi]), WEIGHTS, MULTS)
            res["fraud_prob"], res["confidence"], res["decision"], res["risk"] = fp, conf, dec, risk
            res["seq"] = r["seq"]
        self.scored += m
        return self.torch.from_numpy(res.view(np.uint8).reshape(m, 24).copy())

    def scatter_results(self, res, n, sentinel=False):
        out = R.scatter_results(res.numpy().reshape(-1).view(R.RESULT))
        return tuple(self.torch.from_numpy(a) for a in out)


class StreamingOracleBackend(OracleShardBackend):
    """+ the streaming hooks EngineShardBackend has (forward stream, counts to the host behind an event, records
    scored asynchronously): on the CPU they run inline, so the test checks the protocol — prefetched partitions and
    count exchanges, the records / results exchanges on two process groups — not the streams."""

    def fwd_ctx(self):
        import contextlib
        return contextlib.nullcontext()

    def start_partition(self, txns, n, G, input_ready=None):
        return self.partition(txns, n, G)

    def counts_to_host(self, counts, recv):
        from fdengine.sharding import _HostCounts
        return _HostCounts(self.torch.cat([counts, recv]), None, counts.numel())

    def forward_ready(self):
        return None

    def score_records_async(self, inbox, m, ready):
        return self.score_records(inbox, m)


class AggShardBackend(OracleShardBackend):
    """+ the owner-side keyed aggregates: WindowOracle (windows_ref) and an exact-cents sink (ExactSink), with
    the merchant windows returned as exact-moment partials in the library's fd_merchant_window layout."""

    def __init__(self, *a):
        from oracle.windows_ref import WindowOracle
        super().__init__(*a)
        self.win, self.sink = WindowOracle(), ExactSink()

    def partition(self, txns, n, G, extras=None):
        ex = {k: v.numpy() for k, v in (extras or {}).items()}
        rec, counts = R.partition({k: v.numpy() for k, v in txns.items()}, G, ex.get("payment_method"),
                                  ex.get("is_fraud"))
        t = self.torch
        return t.from_numpy(rec.view(np.uint8).reshape(n, 48).copy()), t.from_numpy(counts)

    def unpack(self, rec, res, m):
        r = rec.numpy().reshape(-1).view(R.RECORD)
        rr = res.numpy().reshape(-1).view(R.RESULT)
        t = self.torch
        return {"card_key": t.from_numpy(r["key"].copy()), "ts_ms": t.from_numpy(r["ts"].copy()),
                "amount_cents": t.from_numpy(r["cents"].copy()), "merchant": t.from_numpy(r["merchant"].copy()),
                "payment_method": t.from_numpy(r["pm"].copy()),
                "is_fraud": t.from_numpy((r["flags"] & 1).astype(np.uint8)),
                "fraud_score": t.from_numpy(rr["fraud_prob"].copy())}

    def windows_observe(self, ts):
        self.win.observe(ts)

    def windows_step(self, cols, m, flush):
        users, merchants = self.win.step(_events(cols), flush)
        return users, merchant_partials(merchants)

    def sink_update(self, cols, m):
        self.sink.update(cols)

    def sink_query(self, kind, buckets, merchants=None):
        return self.sink.query(kind, buckets, merchants)


def _events(cols):
    c = {k: v.numpy() for k, v in cols.items()}
    return [dict(key=int(c["card_key"][i]), ts=int(c["ts_ms"][i]), cents=int(c["amount_cents"][i]),
                 merchant=int(c["merchant"][i]), pm=int(c["payment_method"][i]), fraud=bool(c["is_fraud"][i]),
                 score=float(c["fraud_score"][i])) for i in range(len(c["ts_ms"]))]


def merchant_partials(ms):
    """WindowOracle merchant windows -> fd_merchant_window records (what a shard's device step returns)."""
    from fdengine import _native as N
    out = np.zeros(len(ms), N.MERCHANT_WINDOW_DTYPE)
    for i, w in enumerate(ms):
        for f in ("merchant", "count", "window_start", "window_end", "first_ts", "last_ts", "fraud_count",
                  "high_risk_count", "unique_users", "unique_payment_methods", "total_amount", "fraud_amount",
                  "avg_amount", "fraud_rate", "amount_stddev", "risk_score", "cents", "fraud_cents"):
            out[i][f] = w[f]
        out[i]["sq_lo"] = w["s2"] & (2**64 - 1)
        out[i]["sq_hi"] = w["s2"] >> 64
        mask = [0, 0, 0, 0]
        for pm in w["pm_set"]:
            mask[pm >> 6] |= 1 << (pm & 63)
        out[i]["pm_mask"] = mask
    return out


class ExactSink:
    """RedisTransactionSink.updateAggregations (sink_ref.py) with the engine's declared exact-cents sums:
    per key counts, cents, fraud, high-risk (score > 0.7, hourly) and the distinct users (merchant)."""

    def __init__(self):
        self.t = {}

    def update(self, cols):
        c = {k: v.numpy() for k, v in cols.items()}
        for i in range(len(c["ts_ms"])):
            ts, cents = int(c["ts_ms"][i]), int(c["amount_cents"][i])
            fr, sc = bool(c["is_fraud"][i]), float(c["fraud_score"][i])
            hour, day, m = ts // 3_600_000, ts // 86_400_000, int(c["merchant"][i])
            keys = [(1, -1, hour), (2, -1, day)] + ([(3, m, hour)] if m >= 0 else [])
            for k in keys:
                e = self.t.setdefault(k, [0, 0, 0, 0, set()])
                e[0] += 1
                e[1] += cents
                e[2] += fr
                e[3] += k[0] == 1 and sc == sc and sc > 0.7
                if k[0] == 3:
                    e[4].add(int(c["card_key"][i]) or 1)

    def query(self, kind, buckets, merchants=None):
        from fdengine import _native as N
        out = np.zeros(len(buckets), N.AGGREGATE_DTYPE)
        for i, b in enumerate(buckets):
            e = self.t.get((kind, int(merchants[i]) if kind == 3 else -1, int(b)))
            if e:
                total = e[1] / 100
                out[i] = (e[0], e[2], e[3], len(e[4]), total, e[2] / e[0], total / e[0], 1, 0)
        return out


def _worker(rank, port, outdir, mode="serial"):
    import torch
    import torch.distributed as dist
    from fdengine.sharding import ShardedScorer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        pop, streams = _streams()
        xgb, ifm = _models()
        be = (StreamingOracleBackend if mode != "serial" else OracleShardBackend)(rank, WORLD, pop, xgb, ifm)
        sc = ShardedScorer(be, rank, WORLD)
        assert sc.streaming == (mode != "serial")
        tx = streams[rank]
        outs = []
        parts = [{k: torch.from_numpy(np.ascontiguousarray(v[s * B:(s + 1) * B])) for k, v in tx.items()}
                 for s in range(STEPS)]
        for s in range(STEPS):
            part = parts[s]
            # "prefetch": every step but the last hands over the next batch (and step 2 does not, on every rank)
            pre = (parts[s + 1], B) if mode == "prefetch" and s + 1 < STEPS and s != 2 else None
            fp, conf, dec, risk = sc.step(part, B, prefetch=pre)
            outs.append(np.stack([fp.numpy(), conf.numpy(), dec.numpy().astype(np.float64),
                                  risk.numpy().astype(np.float64)]))
            send, recv = sc.last_counts
            assert sum(send) == B
        np.save(os.path.join(outdir, f"rank{rank}.npy"), np.concatenate(outs, axis=1))
        np.save(os.path.join(outdir, f"scored{rank}.npy"), np.array([be.scored]))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["serial", "streaming", "prefetch"])
def test_world2_gloo_matches_unsharded_oracle(tmp_path, mode):
    """serial: the exchange with a host read of the split sizes; streaming / prefetch: the streaming step (records
    and results on two process groups), prefetch also exchanging the next batch's counts one step ahead"""
    import torch.multiprocessing as mp

    import oracle
    from oracle.features_c import OracleFeatureState
    mp.spawn(_worker, args=(_free_port(), str(tmp_path), mode), nprocs=WORLD, join=True)
    got = [np.load(tmp_path / f"rank{r}.npy") for r in range(WORLD)]
    scored = [int(np.load(tmp_path / f"scored{r}.npy")[0]) for r in range(WORLD)]
    assert sum(scored) == WORLD * B * STEPS and min(scored) > 0  # both owners did work

    # unsharded oracle over the global order: step-major, then ingest rank, then arrival index
    pop, streams = _streams()
    xgb, ifm = _models()
    U, M = pop["users"], pop["merchants"]
    st = OracleFeatureState(4096, 1, 8)
    st.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    st.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    exp = [[] for _ in range(WORLD)]
    for s in range(STEPS):
        for r in range(WORLD):
            part = {k: v[s * B:(s + 1) * B] for k, v in streams[r].items()}
            _, V = st.run(part, want_raw=False)
            px, _, _ = oracle.xgb_predict(xgb, V)
            pi, _, _ = oracle.iforest_predict(ifm, V)
            fp, conf, dec, risk = oracle.blend_weighted(np.stack([px.astype(np.float64), pi]), WEIGHTS, MULTS)
            exp[r].append(np.stack([fp, conf, dec.astype(np.float64), risk.astype(np.float64)]))
    for r in range(WORLD):
        np.testing.assert_array_equal(got[r], np.concatenate(exp[r], axis=1))


# ------------------------------------------------------------------ keyed aggregates across shards (windows, sink)
MF = ("merchant", "window_start", "window_end", "first_ts", "last_ts", "count", "fraud_count", "high_risk_count",
      "unique_users", "unique_payment_methods", "total_amount", "fraud_amount", "avg_amount", "fraud_rate",
      "amount_stddev", "risk_score")
UF = ("user_key", "window_start", "window_end", "first_ts", "last_ts", "count", "fraud_count", "high_risk_count",
      "unique_merchants", "unique_payment_methods", "total_amount", "avg_amount", "fraud_rate", "velocity_score")


def _pm(r):
    rng = np.random.default_rng(90 + r)
    pm = rng.integers(0, 6, B * STEPS).astype(np.uint8)
    pm[rng.random(B * STEPS) < 0.1] = 255
    return pm


def _agg_worker(rank, port, outdir):
    import pickle

    import torch
    import torch.distributed as dist
    from fdengine.sharding import ShardedScorer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        pop, streams = _streams()
        xgb, ifm = _models()
        be = AggShardBackend(rank, WORLD, pop, xgb, ifm)
        sc = ShardedScorer(be, rank, WORLD)
        tx, pm = streams[rank], _pm(rank)
        users, merchants = [], []
        for s in range(STEPS):
            sl = slice(s * B, (s + 1) * B)
            part = {k: torch.from_numpy(np.ascontiguousarray(v[sl])) for k, v in tx.items() if k != "is_fraud"}
            extras = {"payment_method": torch.from_numpy(pm[sl].copy()),
                      "is_fraud": torch.from_numpy(tx["is_fraud"][sl].astype(np.uint8))}
            sc.step(part, B, extras=extras, windows=True, sink=True, flush=s == STEPS - 1)
            uw, mw = sc.last_windows
            users += uw
            merchants.append(mw)
        hours = sorted({int(t) // 3_600_000 for r in range(WORLD) for t in streams[r]["ts_ms"]})
        q = {"hourly": sc.sink_query(1, hours), "daily": sc.sink_query(2, sorted({h // 24 for h in hours}))}
        mids = np.repeat(np.arange(N_MERCH), len(hours))
        q["merchant"] = sc.sink_query(3, np.tile(hours, N_MERCH), mids)
        with open(os.path.join(outdir, f"agg{rank}.pkl"), "wb") as f:
            pickle.dump({"users": users, "merchants": merchants, "sink": q}, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
def test_world2_gloo_windows_and_sink_match_unsharded(tmp_path):
    """Flink window aggregates and sink aggregates under card sharding: one watermark through
    the all-reduce MAX, merchant windows merged from exact-moment partials (fd_merchant_windows_merge), sink
    partials summed at query — against one unsharded run over the global order, field for field."""
    import pickle

    import torch.multiprocessing as mp

    import oracle
    from fdengine import _native as N
    from oracle.features_c import OracleFeatureState
    from oracle.windows_ref import WindowOracle
    mp.spawn(_agg_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    got = [pickle.load(open(tmp_path / f"agg{r}.pkl", "rb")) for r in range(WORLD)]

    pop, streams = _streams()
    xgb, ifm = _models()
    U, M = pop["users"], pop["merchants"]
    st = OracleFeatureState(4096, 1, 8)
    st.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    st.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    win, sink = WindowOracle(), ExactSink()
    exp_users, exp_merch = [], []
    pms = [_pm(r) for r in range(WORLD)]
    for s in range(STEPS):
        evs = []
        for r in range(WORLD):
            sl = slice(s * B, (s + 1) * B)
            part = {k: v[sl] for k, v in streams[r].items()}
            _, V = st.run(part, want_raw=False)
            px, _, _ = oracle.xgb_predict(xgb, V)
            pi, _, _ = oracle.iforest_predict(ifm, V)
            fp, _, _, _ = oracle.blend_weighted(np.stack([px.astype(np.float64), pi]), WEIGHTS, MULTS)
            cols = {"card_key": part["card_key"], "ts_ms": part["ts_ms"], "amount_cents": part["amount_cents"],
                    "merchant": part["merchant"], "payment_method": pms[r][sl],
                    "is_fraud": part["is_fraud"].astype(np.uint8), "fraud_score": fp}
            tcols = {k: __import__("torch").from_numpy(np.ascontiguousarray(v)) for k, v in cols.items()}
            evs += _events(tcols)
            sink.update(tcols)
        uw, mw = win.step(evs, flush=s == STEPS - 1)
        exp_users += uw
        exp_merch += mw
    assert len(exp_merch) > 20 and len(exp_users) > 100  # the windows did fire

    def rows(recs, fields, key):
        return sorted((tuple(r[f].item() if hasattr(r[f], "item") else r[f] for f in fields) for r in recs),
                      key=lambda t: tuple(t[i] for i in key))
    got_users = [u for g in got for u in g["users"]]
    assert rows(got_users, UF, (1, 0)) == rows(exp_users, UF, (1, 0))
    for r in range(WORLD):  # every rank holds the same merged merchant windows
        gm = np.concatenate(got[r]["merchants"])
        assert rows(gm, MF, (1, 0)) == rows(exp_merch, MF, (1, 0))
    for r in range(WORLD):
        q = got[r]["sink"]
        hours = sorted({int(t) // 3_600_000 for rr in range(WORLD) for t in streams[rr]["ts_ms"]})
        np.testing.assert_array_equal(q["hourly"], sink.query(1, hours))
        np.testing.assert_array_equal(q["daily"], sink.query(2, sorted({h // 24 for h in hours})))
        mids = np.repeat(np.arange(N_MERCH), len(hours))
        np.testing.assert_array_equal(q["merchant"], sink.query(3, np.tile(hours, N_MERCH), mids))
        assert q["merchant"]["found"].sum() > 20
    assert N.AGGREGATE_DTYPE  # (dtype in use)
