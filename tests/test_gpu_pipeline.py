"""fd_score_batch_pipelined (the streaming form of fd_score_batch_device: batch i+1's features on the engine's
feature stream overlap batch i's forests) against fd_score_batch_device on a twin engine with the same state:
every batch's outputs bit-identical, the card state after the stream identical (the next batch's vectors), with
other engine calls interleaved and with inputs that arrive on a side stream behind an `input_ready` event. The
pipelined batches that go through the fused ensemble kernel without a vectors output use the compact 64-B row
(fd_internal.h kCompactSlot); the reference engine writes and reads the full 64-wide one: same bits.
Reference chain: FeatureExtractor -> RedisTransactionSink -> FeatureProcessor -> EnsemblePredictor.predict
(fl/features/FeatureExtractor.java:50-87, ml/models/ensemble_predictor.py:75-148), one micro-batch at a time."""
import numpy as np
import pytest

from fdengine import FraudEngine, iforest_from_sklearn, synth, xgboost_from_json_doc
from fdengine._native import TXN_FIELDS

pytestmark = pytest.mark.gpu


def _setup(pop, xgb, ifm, K=16):
    U, M = pop["users"], pop["merchants"]
    eng = FraudEngine(0)
    eng.state_init(1 << 17, 1, K)
    eng.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    eng.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    eng.load_forest(0, xgb)
    eng.load_forest(1, ifm)
    return eng


def _params():
    from oracle import scoring_ref as S
    names = ["xgboost_primary", "isolation_forest"]
    w = S.normalized_weights({"xgboost_primary": 0.4, "isolation_forest": 0.05})
    return FraudEngine.blend_params([w[k] for k in names], [S.CONF_MULT[k] for k in names])


def _outs(n):
    import torch
    return [torch.empty(n, dtype=t, device="cuda") for t in (torch.float64, torch.float64, torch.uint8, torch.uint8)]


@pytest.fixture(scope="module")
def world():
    pop = synth.population(20000, 5000, seed=7)
    tx = synth.txn_stream(pop, 300_000, seed=8)
    warm = FraudEngine(0)
    try:
        U, M = pop["users"], pop["merchants"]
        warm.state_init(1 << 17, 1, 16)
        warm.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
        warm.load_merchants(M["fraud_rate"], M["risk_multiplier"])
        X = warm.features({k: v[:16384] for k, v in tx.items()})
    finally:
        warm.close()
    xgb = xgboost_from_json_doc(synth.xgboost_doc(200, 8, 64, X[-8192:], seed=3))
    ifm = iforest_from_sklearn(synth.isolation_forest(X[-8192:].astype(np.float64), n_estimators=60))
    return pop, tx, xgb, ifm


def _run(world, cuts, interleave=False, side_stream=False, hot=False, lean=1, slot_stream=0, opts=(), K=16):
    import torch
    pop, tx, xgb, ifm = world
    params = _params()
    cols = {f: np.array(tx[f][:cuts[-1]]) for f in TXN_FIELDS}
    if hot:  # batch 1: one card with 2,000 transactions (an oversized bucket), one with 30 (a long segment)
        k = cols["card_key"]
        k[cuts[1]:cuts[2]:20] = k[cuts[1]]
        k[cuts[1] + 7:cuts[1] + 7 + 30 * 97:97] = k[cuts[1] + 7]
    dev = {f: torch.from_numpy(np.ascontiguousarray(cols[f])).cuda() for f in TXN_FIELDS}
    torch.cuda.synchronize()
    ref, pip = _setup(pop, xgb, ifm, K), _setup(pop, xgb, ifm, K)
    pip.set_option("pipeline_lean", lean)
    pip.set_option("slot_stream", slot_stream)
    for k, v in opts:
        pip.set_option(k, v)
    try:
        for e in (ref, pip):
            e.set_stream(torch.cuda.current_stream().cuda_stream)
        got, want = [], []
        side = torch.cuda.Stream() if side_stream else None
        for a, b in zip(cuts[:-1], cuts[1:]):
            n = b - a
            part = {f: t[a:b] for f, t in dev.items()}
            o_ref = _outs(n)
            ref.score_batch_device(params, [0, 1], {f: t.data_ptr() for f, t in part.items()}, n,
                                   *[o.data_ptr() for o in o_ref])
            ev = None
            if side is not None:  # inputs produced on another stream: a fresh copy behind an event
                with torch.cuda.stream(side):
                    part = {f: t.clone() for f, t in part.items()}
                    ev = torch.cuda.Event()
                    ev.record(side)
            o_pip = _outs(n)
            pip.score_batch_pipelined(params, [0, 1], {f: t.data_ptr() for f, t in part.items()}, n,
                                      *[o.data_ptr() for o in o_pip], input_ready=ev.cuda_event if ev else 0)
            if side is not None:
                for t in part.values():
                    t.record_stream(torch.cuda.current_stream())
            if interleave and a == cuts[1]:  # another engine call between two pipelined batches
                for e in (ref, pip):
                    e.load_merchants(pop["merchants"]["fraud_rate"], pop["merchants"]["risk_multiplier"])
            got.append(o_pip)
            want.append(o_ref)
        torch.cuda.synchronize()
        for g, w in zip(got, want):
            for x, y in zip(g, w):
                np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())
        # the card state both engines end with: the next batch's vectors
        nxt = {k: v[cuts[-1]:cuts[-1] + 4096] for k, v in tx.items()}
        np.testing.assert_array_equal(pip.features(nxt), ref.features(nxt))
    finally:
        ref.close()
        pip.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("lean,slot_stream", [(1, 0), (0, 0), (1, 1), (1, 2)])
def test_pipelined_stream_matches_serial(world, lean, slot_stream):
    """slot_stream 1 / 2: every batch's slot pass on the engine's slot stream (high / low priority)"""
    _run(world, [0, 40000, 80000, 81000, 121000, 161000, 201000, 241000], lean=lean, slot_stream=slot_stream)


@pytest.mark.timeout(300)
def test_pipelined_compact_rows_bit_identical_k64(world):
    """The headline's ring capacity (K = 64): the compact 64-B rows (byte-packed integer slots, bins by the
    small-integer table) give the serial 64-wide path's outputs and end state bit for bit, hot cards included
    (the full-size config-4 test checks the compact leg against the oracle at 1e-5 only; a twin engine
    does not fit beside its 155 GB of card pages, so the bit-identity is pinned here)."""
    _run(world, [0, 40000, 80000, 81000, 121000, 161000], hot=True, K=64)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("opts", [(("ensemble_bin_global", 1),), (("lean_group", 0),), (("lean_group", 1),),
                                  (("ensemble_bin_global", 1), ("ensemble_chunks", 2)), (("compact_vectors", 1),),
                                  (("compact_vectors", 1), ("lean_group", 0)), (("compact_vectors", 0),)],
                         ids=["bin_global", "lean_group0", "lean_group1", "bin_global_compact_chunks", "compact64",
                              "compact64_lean_group0", "full_rows"])
def test_pipelined_engine_options(world, opts):
    """the compact path's A/B options (binning of the fused kernel's rows, the lean kernel's card grouping): the
    pipelined stream's outputs and end state equal the serial full-vector path's under every one"""
    _run(world, [0, 40000, 80000, 81000, 121000], hot=True, opts=opts)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("slot_stream", [0, 1])
def test_pipelined_hot_cards_and_events(world, slot_stream):
    """hot-card buckets with inputs behind input_ready events"""
    _run(world, [0, 40000, 80000, 120000, 160000], hot=True, side_stream=True, slot_stream=slot_stream)


@pytest.mark.timeout(300)
def test_pipelined_hot_cards_deferred_buckets(world):
    """buckets the lean kernel cannot take (> 512 keys, a segment > 16) go to the deferred launch"""
    _run(world, [0, 40000, 80000, 120000], hot=True)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("slot_stream", [0, 1])
def test_pipelined_with_interleaved_calls(world, slot_stream):
    _run(world, [0, 40000, 80000, 120000], interleave=True, slot_stream=slot_stream)


@pytest.mark.timeout(300)
def test_pipelined_input_ready_event(world):
    _run(world, [0, 40000, 80000, 120000, 160000], side_stream=True)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("gather", [1, 0])
def test_pipelined_lstm_and_latency_batches(world, gather):
    """models [XGBoost, IsolationForest, LSTM] (the per-model scoring path with the LSTM on its second stream and
    the card histories double-buffered) and latency-size batches (tree-split path): pipelined == serial, model
    columns included. gather 1 (default): batches of <= 4096 transactions take the gather bucket kernel in the
    pipelined step (option pipeline_gather) — a run of them back to back, 4096 and 4097 at the edge"""
    import torch

    from fdengine import lstm as L
    from fdengine._native import FD_SLOT_LSTM
    from oracle import scoring_ref as S
    pop, tx, xgb, ifm = world
    names = ["xgboost_primary", "isolation_forest", "lstm_sequential"]
    w = S.normalized_weights({"xgboost_primary": 0.4, "isolation_forest": 0.05, "lstm_sequential": 0.25})
    params = FraudEngine.blend_params([w[k] for k in names], [S.CONF_MULT[k] for k in names])
    lw = L.random_weights(16, 128, 1, seed=5)
    U, M = pop["users"], pop["merchants"]
    engines = []
    for _ in range(2):
        e = FraudEngine(0)
        e.state_init(1 << 17, 1, 16, seq_len=10)
        e.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
        e.load_merchants(M["fraud_rate"], M["risk_multiplier"])
        e.load_forest(0, xgb)
        e.load_forest(1, ifm)
        e.load_lstm(lw)
        e.set_stream(torch.cuda.current_stream().cuda_stream)
        engines.append(e)
    ref, pip = engines
    pip.set_option("pipeline_gather", gather)
    cuts = [0, 1000, 1700, 2724, 3748, 7844, 11941, 12041, 15000]
    dev = {f: torch.from_numpy(np.ascontiguousarray(tx[f][:cuts[-1]])).cuda() for f in TXN_FIELDS}
    torch.cuda.synchronize()
    try:
        got, want = [], []
        for a, b in zip(cuts[:-1], cuts[1:]):
            n = b - a
            ptrs = {f: t[a:b].data_ptr() for f, t in dev.items()}
            o_ref, o_pip = _outs(n), _outs(n)
            mp_ref = torch.empty((3, n), dtype=torch.float64, device="cuda")
            mp_pip = torch.empty((3, n), dtype=torch.float64, device="cuda")
            ref.score_batch_device(params, [0, 1, FD_SLOT_LSTM], ptrs, n, *[o.data_ptr() for o in o_ref],
                                   model_probs_ptr=mp_ref.data_ptr())
            pip.score_batch_pipelined(params, [0, 1, FD_SLOT_LSTM], ptrs, n, *[o.data_ptr() for o in o_pip],
                                      model_probs_ptr=mp_pip.data_ptr())
            got.append(o_pip + [mp_pip])
            want.append(o_ref + [mp_ref])
        torch.cuda.synchronize()
        for g, w_ in zip(got, want):
            for x, y in zip(g, w_):
                np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())
    finally:
        for e in engines:
            e.close()


@pytest.mark.timeout(300)
def test_pipelined_sharded_scorer_with_windows_and_sink():
    """ShardedScorer at world size 1 over EngineShardBackend(pipelined=True) — the bench's product path — with the
    Flink window aggregates (a5) and the sink aggregates (f3) run on every step's scores: scores, fired user /
    merchant windows and sink queries identical to the same scorer over fd_score_batch_device."""
    import torch

    from fdengine.sharding import EngineShardBackend, ShardedScorer
    pop = synth.population(20000, 80, seed=71)
    B, steps = 40000, 4
    tx = synth.txn_stream(pop, B * steps, seed=72, rate_per_s=20.0)
    rng = np.random.default_rng(80)
    pm = rng.integers(0, 6, B * steps).astype(np.uint8)
    X = synth.feature_matrix(3000, 64, seed=73)
    xgb = xgboost_from_json_doc(synth.xgboost_doc(80, 8, 64, X, seed=74, p_leaf=0.1))
    ifm = iforest_from_sklearn(synth.isolation_forest(X.astype(np.float64), n_estimators=30))
    params = FraudEngine.blend_params([0.4 / 0.45, 0.05 / 0.45], [1.0, 0.5])
    U, M = pop["users"], pop["merchants"]
    dev = {f: torch.from_numpy(np.ascontiguousarray(tx[f])).cuda() for f in TXN_FIELDS}
    extras = {"payment_method": torch.from_numpy(pm).cuda(),
              "is_fraud": torch.from_numpy(tx["is_fraud"].astype(np.uint8)).cuda()}
    torch.cuda.synchronize()
    results, engines = [], []
    try:
        for pipelined in (False, True):
            e = FraudEngine(0)
            engines.append(e)
            e.state_init(1 << 17, 1, 16)
            e.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
            e.load_merchants(M["fraud_rate"], M["risk_multiplier"])
            e.load_forest(0, xgb)
            e.load_forest(1, ifm)
            e.windows_init(1 << 18)
            e.sink_init(1 << 14, 1 << 18)
            sc = ShardedScorer(EngineShardBackend(e, params, [0, 1], pipelined=pipelined), 0, 1)
            scores, users, merchants = [], [], []
            for s in range(steps):
                sl = slice(s * B, (s + 1) * B)
                out = sc.step({f: t[sl] for f, t in dev.items()}, B,
                              extras={k: v[sl] for k, v in extras.items()}, windows=True, sink=True,
                              flush=s == steps - 1)
                scores.append([o.cpu().numpy() for o in out])
                uw, mw = sc.last_windows
                users.append(uw)
                merchants.append(mw)
            hours = sorted({int(t) // 3_600_000 for t in tx["ts_ms"]})
            sink = sc.sink_query(1, hours)
            results.append((scores, users, merchants, sink))
        (s0, u0, m0, k0), (s1, u1, m1, k1) = results
        for a, b in zip(s0, s1):
            for x, y in zip(a, b):
                np.testing.assert_array_equal(x, y)
        # fired windows per step as sets (their order follows card-table slots, which concurrent first inserts
        # of new cards may assign differently)
        for a, b, key in [(x, y, ("user_key", "window_start")) for x, y in zip(u0, u1)] + \
                         [(x, y, ("merchant", "window_start")) for x, y in zip(m0, m1)]:
            assert len(a) == len(b)
            ia, ib = np.lexsort([a[k] for k in key[::-1]]), np.lexsort([b[k] for k in key[::-1]])
            assert bool((a[ia].tobytes() == b[ib].tobytes())), "fired windows differ"
        assert sum(len(w) for w in u0) > 0 and sum(len(w) for w in m0) > 0
        assert bool(k0.tobytes() == k1.tobytes()), "sink aggregates differ"
    finally:
        for e in engines:
            e.close()


@pytest.mark.timeout(300)
def test_pipelined_outputs_dropped_each_step(world):
    """The bench's product path (ShardedScorer at world 1 over EngineShardBackend(pipelined=True)) with a caller that
    keeps nothing on the device: every step's outputs are fresh torch tensors on the engine's stream, each step
    queues a non_blocking D2H of them into pinned host memory and drops them. torch's caching allocator hands the
    freed blocks to the next step at once, so the engine must write the caller's buffers in that stream's order
    (the pipelined call's copy on the engine stream). Results equal the serial fd_score_batch_device bit for bit."""
    import torch

    from fdengine.sharding import EngineShardBackend, ShardedScorer
    pop, tx, xgb, ifm = world
    params = _params()
    cuts = list(range(0, 240_001, 24_000))
    dev = {f: torch.from_numpy(np.ascontiguousarray(tx[f][:cuts[-1]])).cuda() for f in TXN_FIELDS}
    torch.cuda.synchronize()
    ref, pip = _setup(pop, xgb, ifm), _setup(pop, xgb, ifm)
    try:
        sc = ShardedScorer(EngineShardBackend(pip, params, [0, 1], pipelined=True), 0, 1)
        ref.set_stream(torch.cuda.current_stream().cuda_stream)
        got = []
        for a, b in zip(cuts[:-1], cuts[1:]):
            out = sc.step({f: t[a:b] for f, t in dev.items()}, b - a)
            host = [torch.empty(o.shape, dtype=o.dtype, pin_memory=True) for o in out]
            for h, o in zip(host, out):
                h.copy_(o, non_blocking=True)
            del out
            got.append(host)
        torch.cuda.synchronize()
        for (a, b), host in zip(zip(cuts[:-1], cuts[1:]), got):
            o_ref = _outs(b - a)
            ref.score_batch_device(params, [0, 1], {f: t[a:b].data_ptr() for f, t in dev.items()}, b - a,
                                   *[o.data_ptr() for o in o_ref])
            for x, y in zip(host, o_ref):
                np.testing.assert_array_equal(x.numpy(), y.cpu().numpy())
    finally:
        ref.close()
        pip.close()


@pytest.mark.timeout(300)
def test_pipelined_outputs_into_host_mapped_memory(world):
    """ShardedScorer at world 1 (pipelined) with out= buffers in host-mapped pinned memory (hipHostMalloc mapped):
    the engine's output kernel writes the results over PCIe, a ring of 3 output sets reused while steps are in
    flight; every step's results equal the serial fd_score_batch_device bit for bit."""
    import ctypes

    import torch

    from fdengine.sharding import EngineShardBackend, ShardedScorer
    pop, tx, xgb, ifm = world
    params = _params()
    B = 20_000
    cuts = list(range(0, 9 * B + 1, B))
    dev = {f: torch.from_numpy(np.ascontiguousarray(tx[f][:cuts[-1]])).cuda() for f in TXN_FIELDS}
    torch.cuda.synchronize()
    hip = ctypes.CDLL(None)
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    host, sets = [], []
    for _ in range(3):
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        assert hip.hipHostMalloc(ctypes.byref(h), 18 * B + 64, 2) == 0  # hipHostMallocMapped
        assert hip.hipHostGetDevicePointer(ctypes.byref(d), h, 0) == 0
        host.append(h.value)
        sets.append((d.value, d.value + 8 * B, d.value + 16 * B, d.value + 17 * B))

    def view(q, off, ct, k):
        return np.ctypeslib.as_array((ct * k).from_address(host[q] + off)).copy()

    ref, pip = _setup(pop, xgb, ifm), _setup(pop, xgb, ifm)
    try:
        sc = ShardedScorer(EngineShardBackend(pip, params, [0, 1], pipelined=True), 0, 1)
        ref.set_stream(torch.cuda.current_stream().cuda_stream)
        evs, got = [], []
        for j, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
            if j >= 2:  # at most 2 in flight before a set is reused (3 sets)
                evs[j - 2].synchronize()
                q = (j - 2) % 3
                got.append([view(q, 0, ctypes.c_double, B), view(q, 8 * B, ctypes.c_double, B),
                            view(q, 16 * B, ctypes.c_uint8, B), view(q, 17 * B, ctypes.c_uint8, B)])
            res = sc.step({f: t[a:b] for f, t in dev.items()}, b - a, out=sets[j % 3])
            assert res == sets[j % 3]
            ev = torch.cuda.Event()
            ev.record()
            evs.append(ev)
        torch.cuda.synchronize()
        for j in range(len(cuts) - 3, len(cuts) - 1):
            q = j % 3
            got.append([view(q, 0, ctypes.c_double, B), view(q, 8 * B, ctypes.c_double, B),
                        view(q, 16 * B, ctypes.c_uint8, B), view(q, 17 * B, ctypes.c_uint8, B)])
        for (a, b), h in zip(zip(cuts[:-1], cuts[1:]), got):
            o_ref = _outs(b - a)
            ref.score_batch_device(params, [0, 1], {f: t[a:b].data_ptr() for f, t in dev.items()}, b - a,
                                   *[o.data_ptr() for o in o_ref])
            for x, y in zip(h, o_ref):
                np.testing.assert_array_equal(x, y.cpu().numpy())
    finally:
        ref.close()
        pip.close()
        for h in host:
            hip.hipHostFree(h)
