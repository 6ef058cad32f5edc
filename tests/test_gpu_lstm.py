"""GPU parity of the LSTM sequence head (csrc/lstm.hip, f32 MFMA) against the PyTorch fp32 CPU forward
(oracle/lstm_ref.py), tolerance 1e-5 on probabilities (north star), and of the per-card event history
the feature kernel emits for it; then the fused path with the LSTM as a third ensemble model."""
import numpy as np
import pytest

from fdengine import FraudEngine, synth
from fdengine import lstm as L
from fdengine._native import FD_SLOT_LSTM, TXN_FIELDS
from oracle import lstm_ref as R
from oracle.features_c import OracleFeatureState

pytestmark = pytest.mark.gpu

TOL = 1e-5


@pytest.mark.parametrize("n_out", [1, 2])
@pytest.mark.parametrize("n,T", [(1, 10), (15, 10), (16, 1), (17, 16), (1000, 10), (4099, 7)])
def test_lstm_matches_torch(engine, n, T, n_out):
    w = L.random_weights(16, 128, n_out, seed=n + T)
    engine.load_lstm(w)
    rng = np.random.default_rng(n)
    seq = rng.normal(0, 1.5, (n, T, 16)).astype(np.float32)
    p = engine.lstm_predict(seq)
    ref = R.lstm_forward(w, seq)
    assert p.shape == (n,)
    assert np.abs(p - ref).max() <= TOL, np.abs(p - ref).max()


@pytest.mark.parametrize("rows", [4, 16])
@pytest.mark.parametrize("n,T", [(5, 10), (1000, 10), (1029, 13)])
def test_lstm_tile_kernels_match_torch(engine, rows, n, T):
    """both tile forms (4 rows on v_mfma_f32_4x4x1_16b_f32, persistent; 16 rows on 16x16x4) forced through
    the "lstm_rows" option, whatever the batch size"""
    w = L.random_weights(16, 128, 2, seed=3 * n + T)
    engine.load_lstm(w)
    seq = np.random.default_rng(n + 1).normal(0, 1.5, (n, T, 16)).astype(np.float32)
    engine.set_option("lstm_rows", rows)
    try:
        p = engine.lstm_predict(seq)
    finally:
        engine.set_option("lstm_rows", 0)
    assert np.abs(p - R.lstm_forward(w, seq)).max() <= TOL


def test_lstm_narrow_input_and_saturation(engine):
    w = L.random_weights(7, 128, 1, seed=9)
    w.w_hh *= 4.0  # strongly saturating gates
    engine.load_lstm(w)
    seq = np.random.default_rng(2).normal(0, 4.0, (300, 10, 7)).astype(np.float32)
    p = engine.lstm_predict(seq)
    assert np.abs(p - R.lstm_forward(w, seq)).max() <= TOL


@pytest.mark.parametrize("rows", [4, 16])
def test_lstm_non_finite_recurrent_weight(engine, rows):
    """one W_hh weight +inf: PyTorch's step 0 multiplies it by h_{-1} = 0 (NaN), so every probability is NaN; the
    4-row kernel skips step 0's W_hh h_{-1} only when every W_hh weight is finite, so it keeps that NaN too"""
    w = L.random_weights(16, 128, 1, seed=21)
    w.w_hh[5, 3] = np.inf
    engine.load_lstm(w)
    seq = np.random.default_rng(4).normal(0, 1.5, (37, 10, 16)).astype(np.float32)
    engine.set_option("lstm_rows", rows)
    try:
        p = engine.lstm_predict(seq)
    finally:
        engine.set_option("lstm_rows", 0)
    ref = R.lstm_forward(w, seq)
    assert np.isnan(ref).all()
    np.testing.assert_array_equal(np.isnan(p), np.isnan(ref))


def test_lstm_not_loaded_raises(engine):
    engine.unload_lstm()
    with pytest.raises(ValueError):
        engine.lstm_predict(np.zeros((2, 10, 16), np.float32))


def _setup(engine, n_users, T, K=8):
    pop = synth.population(n_users, 100, seed=n_users + 1)
    U, M = pop["users"], pop["merchants"]
    cap = 4 * n_users + 4096
    engine.state_init(cap, 1, K, seq_len=T)
    engine.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    engine.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    orc = OracleFeatureState(cap, 1, K)
    orc.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    orc.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    return pop, orc


def test_feature_kernel_sequences_match_history(engine):
    import torch
    T = 10
    pop, orc = _setup(engine, 300, T)
    tx = synth.txn_stream(pop, 9000, seed=8, rate_per_s=1.0, unknown_user_frac=0.05)
    hist = R.SequenceState(T)
    try:
        engine.set_stream(torch.cuda.current_stream().cuda_stream)
        for a, b in [(0, 1), (1, 700), (700, 9000)]:  # history carried across micro-batches
            n = b - a
            part = {k: v[a:b] for k, v in tx.items()}
            dev = {f: torch.from_numpy(np.ascontiguousarray(part[f])).cuda() for f in TXN_FIELDS}
            vec = torch.empty((n, 64), dtype=torch.float32, device="cuda")
            raw = torch.empty((n, 16), dtype=torch.float64, device="cuda")
            seq = torch.empty((n, T, 16), dtype=torch.float32, device="cuda")
            engine.features_seq_device({f: t.data_ptr() for f, t in dev.items()}, n, vec.data_ptr(), seq.data_ptr(),
                                       raw.data_ptr())
            torch.cuda.synchronize()
            rraw, _ = orc.run(part)
            # oracle history over the oracle's raw features (column 1 may differ by 1 f64 ulp: device log)
            exp = hist.run(part["card_key"], rraw)
            got = seq.cpu().numpy()
            np.testing.assert_array_max_ulp(got, exp, maxulp=1)
            assert (got[:, :, [c for c in range(16) if c != 1]] == exp[:, :, [c for c in range(16) if c != 1]]).all()
    finally:
        engine.set_stream(None)


def test_fused_pipeline_with_lstm(engine):
    """fd_score_batch_device with models [XGBoost, IsolationForest, LSTM]: the LSTM column equals the
    torch forward over the oracle's card histories (<= 1e-5), and the blend uses all three."""
    import torch

    import oracle
    from fdengine import iforest_from_sklearn, xgboost_from_json_doc
    from oracle import scoring_ref as S
    T = 10
    pop, orc = _setup(engine, 2000, T)
    tx = synth.txn_stream(pop, 12000, seed=9, rate_per_s=2.0)
    X = synth.feature_matrix(3000, 64, seed=3)
    xgb = xgboost_from_json_doc(synth.xgboost_doc(80, 8, 64, X, seed=4, p_leaf=0.1))
    ifm = iforest_from_sklearn(synth.isolation_forest(X.astype(np.float64), n_estimators=30))
    lw = L.random_weights(16, 128, 1, seed=5)
    engine.load_forest(0, xgb)
    engine.load_forest(1, ifm)
    engine.load_lstm(lw)
    names = ["xgboost_primary", "isolation_forest", "lstm_sequential"]
    w = S.normalized_weights({"xgboost_primary": 0.4, "isolation_forest": 0.05, "lstm_sequential": 0.25})
    params = FraudEngine.blend_params([w[k] for k in names], [S.CONF_MULT[k] for k in names])
    hist = R.SequenceState(T)
    try:
        engine.set_stream(torch.cuda.current_stream().cuda_stream)
        for a, b in [(0, 5000), (5000, 12000)]:
            n = b - a
            part = {k: v[a:b] for k, v in tx.items()}
            dev = {f: torch.from_numpy(np.ascontiguousarray(part[f])).cuda() for f in TXN_FIELDS}
            out = [torch.empty(n, dtype=d, device="cuda") for d in (torch.float64, torch.float64, torch.uint8,
                                                                     torch.uint8)]
            vec = torch.empty((n, 64), dtype=torch.float32, device="cuda")
            mp = torch.empty((3, n), dtype=torch.float64, device="cuda")
            engine.score_batch_device(params, [0, 1, FD_SLOT_LSTM], {f: t.data_ptr() for f, t in dev.items()}, n,
                                      *[o.data_ptr() for o in out], vec_ptr=vec.data_ptr(),
                                      model_probs_ptr=mp.data_ptr())
            torch.cuda.synchronize()
            rraw, _ = orc.run(part)
            M = mp.cpu().numpy()
            V = vec.cpu().numpy()
            px, _, _ = oracle.xgb_predict(xgb, V)
            pi, _, _ = oracle.iforest_predict(ifm, V)
            pl = R.lstm_forward(lw, hist.run(part["card_key"], rraw))
            assert np.abs(M[0] - px).max() <= TOL and np.abs(M[1] - pi).max() <= TOL
            assert np.abs(M[2] - pl).max() <= TOL, np.abs(M[2] - pl).max()
            fp = out[0].cpu().numpy()
            for i in range(0, n, 11):
                rfp, rcf, _, _ = S.blend_row(names, [float(M[0, i]), float(M[1, i]), float(M[2, i])], w)
                assert fp[i] == rfp
    finally:
        engine.set_stream(None)
        engine.unload_lstm()
