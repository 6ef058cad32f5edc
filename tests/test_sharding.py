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


def _worker(rank, port, outdir):
    import torch
    import torch.distributed as dist
    from fdengine.sharding import ShardedScorer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        pop, streams = _streams()
        xgb, ifm = _models()
        be = OracleShardBackend(rank, WORLD, pop, xgb, ifm)
        sc = ShardedScorer(be, rank, WORLD)
        tx = streams[rank]
        outs = []
        for s in range(STEPS):
            part = {k: torch.from_numpy(np.ascontiguousarray(v[s * B:(s + 1) * B])) for k, v in tx.items()}
            fp, conf, dec, risk = sc.step(part, B)
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
def test_world2_gloo_matches_unsharded_oracle(tmp_path):
    import torch.multiprocessing as mp

    import oracle
    from oracle.features_c import OracleFeatureState
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
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
