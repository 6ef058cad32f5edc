"""Latency batches (fd_score_batch_device, < 128 tiles: the tree-split forests, the LSTM on 4-transaction tiles):
the engine options small_streams (side streams for the LSTM / the second forest) and seq_ring_lstm give the same
outputs bit for bit, and the split path's per-tile NaN flags are per call (a NaN batch never leaks into the next).
Reference chain: FeatureExtractor -> FeatureProcessor -> EnsemblePredictor.predict one micro-batch at a time
(fl/features/FeatureExtractor.java:50-87, ml/models/ensemble_predictor.py:75-148)."""
import numpy as np
import pytest

from fdengine import FraudEngine, iforest_from_sklearn, synth, xgboost_from_json_doc
from fdengine import lstm as L
from fdengine._native import FD_SLOT_LSTM, TXN_FIELDS

pytestmark = pytest.mark.gpu


def _params(lstm):
    from oracle import scoring_ref as S
    names = ["xgboost_primary", "isolation_forest"] + (["lstm_sequential"] if lstm else [])
    w = S.normalized_weights({"xgboost_primary": 0.4, "isolation_forest": 0.05, "lstm_sequential": 0.3})
    return FraudEngine.blend_params([w[k] for k in names], [S.CONF_MULT[k] for k in names])


def _setup(pop, xgb, ifm, lw):
    U, M = pop["users"], pop["merchants"]
    eng = FraudEngine(0)
    eng.state_init(1 << 17, 1, 16, seq_len=10 if lw is not None else 0)
    eng.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    eng.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    eng.load_forest(0, xgb)
    eng.load_forest(1, ifm)
    if lw is not None:
        eng.load_lstm(lw)
    return eng


@pytest.fixture(scope="module")
def world():
    pop = synth.population(20000, 5000, seed=11)
    tx = synth.txn_stream(pop, 120_000, seed=12)
    X = synth.feature_matrix(8192, 64, seed=13)
    xgb = xgboost_from_json_doc(synth.xgboost_doc(120, 8, 64, X, seed=14))
    ifm = iforest_from_sklearn(synth.isolation_forest(X.astype(np.float64), n_estimators=40))
    return pop, tx, xgb, ifm


@pytest.mark.timeout(200)
def test_small_streams_variants_identical(world):
    """engine option small_streams (latency batches: the LSTM and the second forest on 2 / 1 / 0 side streams) and,
    on one stream, latency_fused (1: both walks in one launch, both sums + the blend in another; 0: per-forest walk
    and sum launches + the blend kernel): the same outputs bit for bit, batch after batch"""
    import torch
    pop, tx, xgb, ifm = world
    lw = L.random_weights(seed=6)
    params = _params(True)
    slots = [0, 1, FD_SLOT_LSTM]
    dev = {f: torch.from_numpy(np.ascontiguousarray(tx[f][:8000])).cuda() for f in TXN_FIELDS}
    engs = [_setup(pop, xgb, ifm, lw) for _ in range(4)]
    try:
        res = []
        for v, e in enumerate(engs):
            e.set_option("small_streams", v if v < 3 else 0)
            e.set_option("latency_fused", 0 if v == 3 else 1)
            e.set_stream(torch.cuda.current_stream().cuda_stream)
            out = []
            for a in range(0, 8000, 1000):
                fp, conf = (torch.empty(1000, dtype=torch.float64, device="cuda") for _ in range(2))
                dec, risk = (torch.empty(1000, dtype=torch.uint8, device="cuda") for _ in range(2))
                mp = torch.empty((3, 1000), dtype=torch.float64, device="cuda")
                e.score_batch_device(params, slots, {f: t[a:a + 1000].data_ptr() for f, t in dev.items()}, 1000,
                                     fp.data_ptr(), conf.data_ptr(), dec.data_ptr(), risk.data_ptr(),
                                     model_probs_ptr=mp.data_ptr())
                out.append([fp, conf, dec, risk, mp])
            res.append(out)
        torch.cuda.synchronize()
        for v in (1, 2, 3):
            for b, (x, y) in enumerate(zip(res[v], res[0])):
                for s, t in zip(x, y):
                    assert np.array_equal(s.cpu().numpy(), t.cpu().numpy()), f"variant {v} batch {b}"
    finally:
        for e in engs:
            e.close()


@pytest.mark.timeout(200)
def test_split_path_nan_flags_per_call(world):
    """The tree-split path's per-tile "holds a NaN" flags are set by the binning launch and cleared by the step's own
    sum kernel (no host-side epoch that one call could compare against a stale value of). Scoring vectors from the
    feature kernel are always finite (FeatureProcessor's final validation), so NaN reaches this path through
    fd_score_matrix / predict: latency batches alternating with and without NaN (and NaN in a single tile), each
    equal to the oracle (leaf ids exact, XGBoost `x < thr` with NaN -> default direction, sklearn NaN rows)."""
    import oracle
    _, _, xgb, ifm = world
    eng = FraudEngine(0)
    try:
        eng.load_forest(0, xgb)
        eng.load_forest(1, ifm)
        for i in range(8):
            X = synth.feature_matrix(1000, 64, seed=40 + i, nan_frac=0.05 if i % 2 == 0 else 0.0)
            if i == 3:
                X[700, 5] = np.nan  # one NaN in the third tile only
            px, mx, lx = eng.predict(0, X, want_raw=True, want_leaf=True)
            rpx, rmx, rlx = oracle.xgb_predict(xgb, X, want_leaf=True)
            assert (lx == rlx).all() and (mx.astype(np.float32) == rmx).all(), f"XGBoost call {i}"
            pi, di, li = eng.predict(1, X, want_raw=True, want_leaf=True)
            rpi, rdi, rli = oracle.iforest_predict(ifm, X, want_leaf=True)
            assert (li == rli).all() and (di == rdi).all(), f"IsolationForest call {i}"
    finally:
        eng.close()


@pytest.mark.timeout(200)
@pytest.mark.parametrize("strategy", [0, 1, 2])
def test_latency_fused_pair_matches_per_forest_path(world, strategy):
    """XGBoost + IsolationForest on 1 k matrices with NaNs (fd_score_matrix, the latency split path): the fused pair
    (latency_fused 1) equals the per-forest launches + blend kernel (0) bit for bit — model probabilities, fraud
    probability, confidence, decision, risk — for every blend strategy, and the model probabilities equal the oracle
    within 1e-5 (leaf sums exact)."""
    import oracle
    _, _, xgb, ifm = world
    from oracle import scoring_ref as S
    names = ["xgboost_primary", "isolation_forest"]
    w = S.normalized_weights({"xgboost_primary": 0.4, "isolation_forest": 0.05})
    params = FraudEngine.blend_params([w[k] for k in names], [S.CONF_MULT[k] for k in names], strategy=strategy)
    eng = FraudEngine(0)
    try:
        eng.load_forest(0, xgb)
        eng.load_forest(1, ifm)
        for i in range(4):
            X = synth.feature_matrix(1000 + 37 * i, 64, seed=60 + i, nan_frac=0.02 if i % 2 == 0 else 0.0)
            eng.set_option("latency_fused", 1)
            a = eng.score_matrix(params, [0, 1], X)
            eng.set_option("latency_fused", 0)
            b = eng.score_matrix(params, [0, 1], X)
            for x, y in zip(a, b):
                np.testing.assert_array_equal(x, y)
            px, _, _ = oracle.xgb_predict(xgb, X)
            pi, _, _ = oracle.iforest_predict(ifm, X)
            assert np.abs(a[0][0] - px).max() <= 1e-5 and np.abs(a[0][1] - pi).max() <= 1e-12
    finally:
        eng.close()


@pytest.mark.timeout(200)
@pytest.mark.parametrize("users", [50, 3000])
def test_lstm_ring_sequences_identical(world, users):
    """Latency batches read each card's last transaction's LSTM sequence from the card's history ring (engine
    option seq_ring_lstm 1, descriptors from the feature kernel) instead of a materialised copy (0): the same model
    probabilities and outputs bit for bit, batch after batch — including cards repeated inside a batch (their earlier
    transactions' sequences materialised), hot cards on the cooperative path (50 users: ~20 transactions per card per
    batch), short histories (left padding) and ragged batch sizes."""
    import torch
    _, _, xgb, ifm = world
    pop = synth.population(users, 500, seed=70 + users)
    tx = synth.txn_stream(pop, 6000, seed=71, rate_per_s=50.0)
    lw = L.random_weights(seed=7)
    params = _params(True)
    slots = [0, 1, FD_SLOT_LSTM]
    dev = {f: torch.from_numpy(np.ascontiguousarray(tx[f])).cuda() for f in TXN_FIELDS}
    engs = [_setup(pop, xgb, ifm, lw) for _ in range(2)]
    sizes = [1, 1000, 997, 1000, 1024, 1978]
    try:
        res = []
        for v, e in enumerate(engs):
            e.set_option("seq_ring_lstm", v)
            e.set_stream(torch.cuda.current_stream().cuda_stream)
            out, a = [], 0
            for B in sizes:
                fp, conf = (torch.empty(B, dtype=torch.float64, device="cuda") for _ in range(2))
                dec, risk = (torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(2))
                mp = torch.empty((3, B), dtype=torch.float64, device="cuda")
                e.score_batch_device(params, slots, {f: t[a:a + B].data_ptr() for f, t in dev.items()}, B,
                                     fp.data_ptr(), conf.data_ptr(), dec.data_ptr(), risk.data_ptr(),
                                     model_probs_ptr=mp.data_ptr())
                out.append([fp, conf, dec, risk, mp])
                a += B
            res.append(out)
        torch.cuda.synchronize()
        for b, (x, y) in enumerate(zip(res[1], res[0])):
            for s, t in zip(x, y):
                assert np.array_equal(s.cpu().numpy(), t.cpu().numpy()), f"batch {b}"
    finally:
        for e in engs:
            e.close()


@pytest.mark.timeout(200)
@pytest.mark.parametrize("users", [50, 3000])
def test_slot_gather_identical(world, users):
    """Batches of <= 4096 transactions find their card slots inside the bucket kernel (engine option slot_gather 1:
    each bucket workgroup takes the keys that hash to it, no slot launch) instead of the slot kernel first (0): the
    same outputs bit for bit, batch after batch, and the same card state after them (the next batch's vectors) —
    hot cards (50 users: ~80 transactions per card per 4 k batch), new cards inserted inside the bucket kernel,
    a batch of 1, the 4096 limit and one past it."""
    import torch
    _, _, xgb, ifm = world
    pop = synth.population(users, 500, seed=90 + users)
    tx = synth.txn_stream(pop, 16000, seed=91, rate_per_s=50.0)
    lw = L.random_weights(seed=7)
    params = _params(True)
    slots = [0, 1, FD_SLOT_LSTM]
    dev = {f: torch.from_numpy(np.ascontiguousarray(tx[f])).cuda() for f in TXN_FIELDS}
    engs = [_setup(pop, xgb, ifm, lw) for _ in range(2)]
    sizes = [1, 1000, 997, 4096, 4097, 1024]
    try:
        res = []
        for v, e in enumerate(engs):
            e.set_option("slot_gather", v)
            e.set_stream(torch.cuda.current_stream().cuda_stream)
            out, a = [], 0
            for B in sizes:
                fp, conf = (torch.empty(B, dtype=torch.float64, device="cuda") for _ in range(2))
                dec, risk = (torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(2))
                mp = torch.empty((3, B), dtype=torch.float64, device="cuda")
                e.score_batch_device(params, slots, {f: t[a:a + B].data_ptr() for f, t in dev.items()}, B,
                                     fp.data_ptr(), conf.data_ptr(), dec.data_ptr(), risk.data_ptr(),
                                     model_probs_ptr=mp.data_ptr())
                out.append([fp, conf, dec, risk, mp])
                a += B
            res.append(out)
        torch.cuda.synchronize()
        for b, (x, y) in enumerate(zip(res[1], res[0])):
            for s, t in zip(x, y):
                assert np.array_equal(s.cpu().numpy(), t.cpu().numpy()), f"batch {b}"
        nxt = {k: v[sum(sizes):sum(sizes) + 2000] for k, v in tx.items()}
        np.testing.assert_array_equal(engs[1].features(nxt), engs[0].features(nxt))
    finally:
        for e in engs:
            e.close()


@pytest.mark.timeout(200)
@pytest.mark.parametrize("lstm,mode", [(True, 1), (True, 2), (True, 3), (False, 1)])
def test_prebin_in_lstm_launch_identical(world, lstm, mode):
    """Latency batches bin the XGBoost + IsolationForest pair's vectors for the tree-split walks in workgroups of the
    LSTM head's launch, ahead of its own (engine option latency_prebin 1) or after them (2), or inside the LSTM's own
    workgroups a lifting level per recurrence step (3; a batch of 1 falls back to 2) — no binning launch —, instead of
    split_bin_pair_kernel (0): the same outputs bit for bit, batch after batch — vectors also written to the caller's
    buffer, ragged sizes (a tile's padding rows), a batch of 1, and the sizes where the 16-row LSTM kernel runs
    (4096, 4097: the binning launch). The engine counter latency_prebinned_batches counts the pair launches that used
    the LSTM launch's bins; without the LSTM head there are none (the binning launch stays)."""
    import torch
    _, _, xgb, ifm = world
    pop = synth.population(3000, 500, seed=95)
    tx = synth.txn_stream(pop, 16000, seed=96, rate_per_s=50.0)
    lw = L.random_weights(seed=8) if lstm else None
    params = _params(lstm)
    slots = [0, 1, FD_SLOT_LSTM] if lstm else [0, 1]
    dev = {f: torch.from_numpy(np.ascontiguousarray(tx[f])).cuda() for f in TXN_FIELDS}
    engs = [_setup(pop, xgb, ifm, lw) for _ in range(2)]
    sizes = [1, 1000, 997, 4096, 4097, 1024, 300]
    try:
        res = []
        for v, e in enumerate(engs):
            e.set_option("latency_prebin", mode if v else 0)
            e.set_stream(torch.cuda.current_stream().cuda_stream)
            out, a = [], 0
            for k, B in enumerate(sizes):
                fp, conf = (torch.empty(B, dtype=torch.float64, device="cuda") for _ in range(2))
                dec, risk = (torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(2))
                mp = torch.empty((len(slots), B), dtype=torch.float64, device="cuda")
                vec = torch.empty((B, 64), dtype=torch.float32, device="cuda") if k % 2 else None
                e.score_batch_device(params, slots, {f: t[a:a + B].data_ptr() for f, t in dev.items()}, B,
                                     fp.data_ptr(), conf.data_ptr(), dec.data_ptr(), risk.data_ptr(),
                                     model_probs_ptr=mp.data_ptr(), vec_ptr=vec.data_ptr() if vec is not None else 0)
                out.append([fp, conf, dec, risk, mp] + ([vec] if vec is not None else []))
                a += B
            res.append(out)
        torch.cuda.synchronize()
        for b, (x, y) in enumerate(zip(res[1], res[0])):
            for s, t in zip(x, y):
                assert np.array_equal(s.cpu().numpy(), t.cpu().numpy()), f"batch {b}"
        assert engs[0].counter("latency_prebinned_batches") == 0
        assert engs[1].counter("latency_prebinned_batches") == (sum(B < 4096 for B in sizes) if lstm else 0)
    finally:
        for e in engs:
            e.close()
