"""GPU: card-hash routing kernels (csrc/route.hip) and the sharded hot path.

* fd_route_partition_device == oracle/route_ref.partition byte for byte (records incl. padding, counts),
  ragged sizes and 1..64 shards;
* fd_route_scatter_results_device inverts any permutation of result records;
* a G-shard step emulated on one GPU (G engines, each owning its cards' state; the all-to-alls done
  by slicing) gives bit-identical results to one unsharded engine over the global arrival order
  (step, ingest rank, index) — the unsharded fused path is itself checked against the oracle in
  test_gpu_features.py::test_fused_pipeline_matches_oracle_chain — and the oracle chain agrees within
  the north-star tolerance (1e-5)."""
import numpy as np
import pytest

from fdengine import FraudEngine, synth
from fdengine._native import TXN_FIELDS
from oracle import route_ref as R

pytestmark = pytest.mark.gpu


def _dev(part):
    import torch
    return {f: torch.from_numpy(np.ascontiguousarray(part[f])).cuda() for f in TXN_FIELDS}


@pytest.mark.parametrize("n", [0, 1, 255, 257, 4099, 65536])
@pytest.mark.parametrize("G", [1, 2, 3, 8, 64])
def test_partition_matches_oracle(engine, n, G):
    import torch
    pop = synth.population(3000, 100, seed=7)
    tx = synth.txn_stream(pop, max(n, 1), seed=n + G, rate_per_s=10.0)
    tx = {k: v[:n] for k, v in tx.items()}
    from fdengine.sharding import EngineShardBackend
    be = EngineShardBackend(engine, FraudEngine.blend_params([1.0], [1.0]), [0])
    engine.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        rec, counts = be.partition(_dev(tx), n, G)
        torch.cuda.synchronize()
    finally:
        engine.set_stream(None)
    rrec, rcounts = R.partition(tx, G)
    np.testing.assert_array_equal(counts.cpu().numpy(), rcounts)
    assert rec.cpu().numpy().tobytes() == rrec.tobytes()


def test_scatter_results_inverts_permutation(engine):
    import torch
    n = 70001
    rng = np.random.default_rng(3)
    res = np.zeros(n, R.RESULT)
    res["fraud_prob"] = rng.random(n)
    res["confidence"] = rng.random(n)
    res["decision"] = rng.integers(0, 4, n)
    res["risk"] = rng.integers(0, 5, n)
    res["seq"] = rng.permutation(n).astype(np.uint32)
    d = torch.from_numpy(res.view(np.uint8).copy()).cuda()
    outs = [torch.empty(n, dtype=t, device="cuda") for t in (torch.float64, torch.float64, torch.uint8, torch.uint8)]
    engine.route_scatter_results_device(d.data_ptr(), n, *[o.data_ptr() for o in outs])
    engine.sync()
    for got, exp in zip(outs, R.scatter_results(res)):
        np.testing.assert_array_equal(got.cpu().numpy(), exp)


def test_scatter_rejects_foreign_records(engine):
    import torch
    res = np.zeros(4, R.RESULT)
    res["seq"] = [0, 1, 2, 9]  # 9 is outside a 4-record batch
    d = torch.from_numpy(res.view(np.uint8).copy()).cuda()
    fp = torch.empty(4, dtype=torch.float64, device="cuda")
    engine.route_scatter_results_device(d.data_ptr(), 4, fp.data_ptr())
    with pytest.raises(Exception) as ei:
        engine.sync()
    assert "outside its micro-batch" in str(ei.value)


@pytest.mark.parametrize("G", [2, 3])
def test_emulated_shards_match_unsharded(G):
    import torch

    import oracle
    from fdengine import iforest_from_sklearn, xgboost_from_json_doc
    from fdengine.sharding import EngineShardBackend
    from oracle.features_c import OracleFeatureState
    n_users, B, steps = 3000, 6000, 3
    pop = synth.population(n_users, 200, seed=17)
    U, M = pop["users"], pop["merchants"]
    streams = [synth.txn_stream(pop, B * steps, seed=60 + r, rate_per_s=4.0) for r in range(G)]
    X = synth.feature_matrix(4000, 64, seed=5)
    xgb = xgboost_from_json_doc(synth.xgboost_doc(120, 8, 64, X, seed=6, p_leaf=0.1))
    ifm = iforest_from_sklearn(synth.isolation_forest(X.astype(np.float64), n_estimators=40))
    w, mult = [0.4 / 0.45, 0.05 / 0.45], [1.0, 0.5]
    params = FraudEngine.blend_params(w, mult)
    stream = torch.cuda.current_stream().cuda_stream

    def make_engine(owned):
        e = FraudEngine(0)
        e.set_stream(stream)
        e.state_init(4 * n_users + 1024, 1, 8)
        e.load_users(U["key"][owned], U["avg_amount"][owned], U["account_age_days"][owned], U["device_fp"][owned])
        e.load_merchants(M["fraud_rate"], M["risk_multiplier"])
        e.load_forest(0, xgb)
        e.load_forest(1, ifm)
        return e

    own = R.shard_of(U["key"], G)
    engines = [make_engine(own == r) for r in range(G)]
    ref = make_engine(np.ones(n_users, bool))
    bes = [EngineShardBackend(e, params, [0, 1]) for e in engines]
    orc = OracleFeatureState(4 * n_users + 1024, 1, 8)
    orc.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    orc.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    try:
        for s in range(steps):
            parts = [{k: v[s * B:(s + 1) * B] for k, v in streams[r].items()} for r in range(G)]
            devs = [_dev(p) for p in parts]
            # 1. partition on every ingest GPU
            out = [be.partition(d, B, G) for be, d in zip(bes, devs)]
            cnts = [c.cpu().numpy() for _, c in out]
            offs = [np.concatenate([[0], np.cumsum(c)]) for c in cnts]
            # 2-3. all-to-all of records: owner o receives sources in rank order
            inbox = [torch.cat([out[src][0][offs[src][o]:offs[src][o + 1]] for src in range(G)]) for o in range(G)]
            # 4. owners score
            res = [bes[o].score_records(inbox[o], len(inbox[o])) for o in range(G)]
            # 5. all-to-all back: source src gets its slice from each owner, in owner order
            roff = [np.concatenate([[0], np.cumsum([cnts[src][o] for src in range(G)])]) for o in range(G)]
            back = [torch.cat([res[o][roff[o][src]:roff[o][src + 1]] for o in range(G)]) for src in range(G)]
            # 6. scatter back to arrival order
            got = [bes[r].scatter_results(back[r], B) for r in range(G)]
            # unsharded reference: one engine over the global order (rank-major inside the step)
            for r in range(G):
                fp = torch.empty(B, dtype=torch.float64, device="cuda")
                cf = torch.empty(B, dtype=torch.float64, device="cuda")
                dc = torch.empty(B, dtype=torch.uint8, device="cuda")
                rk = torch.empty(B, dtype=torch.uint8, device="cuda")
                vec = torch.empty((B, 64), dtype=torch.float32, device="cuda")
                ref.score_batch_device(params, [0, 1], {f: t.data_ptr() for f, t in devs[r].items()}, B, fp.data_ptr(),
                                       cf.data_ptr(), dc.data_ptr(), rk.data_ptr(), vec_ptr=vec.data_ptr())
                torch.cuda.synchronize()
                for a, b in zip(got[r], (fp, cf, dc, rk)):
                    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
                # and the oracle chain on the same global order
                _, V = orc.run(parts[r], want_raw=False)
                px, _, _ = oracle.xgb_predict(xgb, V)
                pi, _, _ = oracle.iforest_predict(ifm, V)
                rfp, _, _, _ = oracle.blend_weighted(np.stack([px.astype(np.float64), pi]), w, mult)
                assert np.abs(got[r][0].cpu().numpy() - rfp).max() <= 1e-5
        for e in engines:
            e.sync()
    finally:
        for e in engines + [ref]:
            e.close()


@pytest.mark.timeout(300)
def test_streaming_routed_step_single_rank_matches_direct():
    """The sharded step's own GPU work on one GPU (ShardedScorer(force_route=True) over a 1-rank RCCL process group),
    in both streaming forms — native: one fd_sharded_step per batch over the engine's own RCCL communicators
    (grouped ncclSend/ncclRecv of counts, records and results, or the counts as one ncclAllGather; the next batch's
    counts one step ahead, named by id; a prefetch of the wrong batch is dropped);
    python: fd_route_partition_stream + torch.distributed all-to-alls on two groups + fd_score_records_pipelined —
    each step's device outputs dropped at once, bit-identical to the direct pipelined step (fd_score_batch_pipelined)
    on a twin engine."""
    import socket

    import torch
    import torch.distributed as dist

    from fdengine import iforest_from_sklearn, xgboost_from_json_doc
    from fdengine.sharding import EngineShardBackend, ShardedScorer
    pop = synth.population(30000, 500, seed=61)
    B, steps = 50000, 6
    tx = synth.txn_stream(pop, B * steps, seed=62, rate_per_s=20.0)
    X = synth.feature_matrix(4000, 64, seed=63)
    xgb = xgboost_from_json_doc(synth.xgboost_doc(120, 8, 64, X, seed=64))
    ifm = iforest_from_sklearn(synth.isolation_forest(X.astype(np.float64), n_estimators=40))
    params = FraudEngine.blend_params([0.4 / 0.45, 0.05 / 0.45], [1.0, 0.5])
    U, M = pop["users"], pop["merchants"]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    engines = []
    ring = None
    try:
        dev = _dev(tx)
        parts = [{f: t[i * B:(i + 1) * B] for f, t in dev.items()} for i in range(steps)]
        torch.cuda.synchronize()
        res = []
        for variant in ("direct", "native", "native_gather", "native_hostout", "python"):
            routed = variant != "direct"
            e = FraudEngine(0)
            engines.append(e)
            if variant == "native_gather":  # the counts as one ncclAllGather (the default from 4 ranks) on real RCCL
                e.set_option("count_exchange", 1)
            e.state_init(1 << 17, 1, 16)
            e.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
            e.load_merchants(M["fraud_rate"], M["risk_multiplier"])
            e.load_forest(0, xgb)
            e.load_forest(1, ifm)
            sc = ShardedScorer(EngineShardBackend(e, params, [0, 1], pipelined=True), 0, 1, force_route=routed,
                               native=None if variant != "python" else False)
            assert sc.streaming == routed and sc.native == variant.startswith("native")
            outs = []
            for i in range(steps):
                pre = (parts[i + 1], B) if i + 1 < steps and i != 3 else None  # one step without prefetch
                if i == 1 and variant.startswith("native"):  # a prefetched batch that is not the next one: dropped
                    pre = (parts[3], B)
                if variant == "native_hostout":  # outputs straight into host-mapped pinned memory (bench loaded loop)
                    if ring is None:
                        import bench
                        ring = bench.HostOutRing(B, steps)
                    sc.step(parts[i], B, prefetch=pre, out=ring.sets[i])
                    outs.append(i)
                    continue
                out = sc.step(parts[i], B, prefetch=pre)
                host = [torch.empty(o.shape, dtype=o.dtype, pin_memory=True) for o in out]
                for h, o in zip(host, out):
                    h.copy_(o, non_blocking=True)
                outs.append(host)
            torch.cuda.synchronize()
            if routed:
                assert sc.last_counts == ([B], [B])
            if variant == "native_hostout":
                import ctypes
                outs = []
                for i in range(steps):
                    h = ring.host[i]
                    col = lambda off, ct: np.ctypeslib.as_array((ct * B).from_address(h + off)).copy()
                    outs.append([torch.from_numpy(col(0, ctypes.c_double)), torch.from_numpy(col(8 * B, ctypes.c_double)),
                                 torch.from_numpy(col(16 * B, ctypes.c_uint8)),
                                 torch.from_numpy(col(17 * B, ctypes.c_uint8))])
            res.append(outs)
        for other in res[1:]:
            for a, b in zip(res[0], other):
                for x, y in zip(a, b):
                    np.testing.assert_array_equal(x.numpy(), y.numpy())
    finally:
        for e in engines:
            e.close()
        if ring is not None:
            ring.close()
        dist.destroy_process_group()
