"""GPU parity of the feature kernels (fd_features_*) against the CPU oracle on the same seeded stream:
bridged raw features bit-exact (counts are integers, sums integer cents / 100.0), scoring vectors
bit-exact except transcendental slots, which may differ by at most 1 f32 ulp (device log1p vs libm),
state carried across micro-batches, both window modes, repeat cards inside a batch (arrival order),
unknown users / merchants."""
import numpy as np
import pytest

from fdengine import FraudEngine, synth
from oracle import velocity_ref as VR
from oracle.features_c import OracleFeatureState

pytestmark = pytest.mark.gpu


def _pair(engine, mode, n_users, n_merch=200, K=8, cap=None):
    pop = synth.population(n_users, n_merch, seed=n_users)
    U, M = pop["users"], pop["merchants"]
    cap = cap or 4 * n_users + 4096
    engine.state_init(cap, mode, K)
    engine.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    engine.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    orc = OracleFeatureState(cap, mode, K)
    orc.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    orc.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    return pop, orc


def _slice(tx, a, b):
    return {k: v[a:b] for k, v in tx.items()}


def _check_raw(raw, rraw):
    """Exact except column 1 (Java Math.log(amount + 1)): device log vs libm, <= 1 f64 ulp."""
    cols = [c for c in range(raw.shape[1]) if c != 1]
    np.testing.assert_array_equal(raw[:, cols], rraw[:, cols])
    np.testing.assert_array_max_ulp(raw[:, 1], rraw[:, 1], maxulp=1)


def _check_vectors(vec, rvec):
    same = vec == rvec
    if not same.all():
        bad = np.argwhere(~same)
        assert set(bad[:, 1].tolist()) <= {1}, f"non-transcendental slots differ: {sorted(set(bad[:, 1].tolist()))}"
        ulps = np.abs(vec.view(np.int32)[~same].astype(np.int64) - rvec.view(np.int32)[~same].astype(np.int64))
        assert ulps.max() <= 1


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("n_users,rate", [(200, 0.5), (20000, 50.0)])  # dense repeats / mostly distinct
def test_features_match_oracle_across_batches(engine, mode, n_users, rate):
    pop, orc = _pair(engine, mode, n_users)
    tx = synth.txn_stream(pop, 24000, seed=3, rate_per_s=rate, unknown_user_frac=0.03, unknown_merchant_frac=0.03)
    for a, b in [(0, 1), (1, 257), (257, 8000), (8000, 24000)]:  # ragged micro-batches, state carried
        part = _slice(tx, a, b)
        vec, raw = engine.features(part, want_raw=True)
        rraw, rvec = orc.run(part)
        _check_raw(raw, rraw)
        _check_vectors(vec, rvec)
    info = engine.state_info()
    assert info["cards"] >= n_users


def test_small_stream_against_python_chain(engine):
    """The pinned chain itself (Java restatement -> FeatureProcessor restatement) on a small stream."""
    pop = synth.population(60, 20, seed=9)
    U, M = pop["users"], pop["merchants"]
    engine.state_init(1024, 0, 1)
    engine.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    engine.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    py = VR.FeatureState(0)
    py.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    py.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    tx = synth.txn_stream(pop, 600, seed=10, rate_per_s=0.2)
    vec, raw = engine.features(tx, want_raw=True)
    rraw = py.run(tx)
    _check_raw(raw, rraw)
    _check_vectors(vec, VR.vectors(rraw).astype(np.float32))


def test_table_full_is_reported(engine):
    engine.state_init(8, 0, 1)
    pop = synth.population(4, 2, seed=1)
    tx = synth.txn_stream(pop, 64, seed=2, unknown_user_frac=1.0)  # 64 distinct unknown cards > 8 slots
    with pytest.raises(Exception) as ei:
        engine.features(tx)
    assert "card table full" in str(ei.value)


def test_fused_pipeline_matches_oracle_chain(engine):
    """fd_score_batch_device (features -> XGBoost + IsolationForest -> blend) == oracle chain."""
    import torch
    import oracle
    from oracle import scoring_ref as S
    from fdengine import iforest_from_sklearn, xgboost_from_json_doc
    from fdengine._native import DECISIONS, RISK_LEVELS, TXN_FIELDS
    pop, orc = _pair(engine, 0, 5000)
    tx = synth.txn_stream(pop, 20000, seed=4, rate_per_s=5.0)
    # models on realistic vectors (a warm-up slice through the oracle state)
    orc_ref = OracleFeatureState(1 << 15, 0, 1)
    orc_ref.load_users(pop["users"]["key"], pop["users"]["avg_amount"], pop["users"]["account_age_days"],
                       pop["users"]["device_fp"])
    orc_ref.load_merchants(pop["merchants"]["fraud_rate"], pop["merchants"]["risk_multiplier"])
    _, Xref = orc_ref.run(tx)
    xgb = xgboost_from_json_doc(synth.xgboost_doc(150, 8, 64, Xref[:4096], seed=6, p_leaf=0.1))
    ifm = iforest_from_sklearn(synth.isolation_forest(Xref[:4096].astype(np.float64)))
    engine.load_forest(0, xgb)
    engine.load_forest(1, ifm)
    names = ["xgboost_primary", "isolation_forest"]
    w = S.normalized_weights({"xgboost_primary": 0.4, "isolation_forest": 0.05})
    params = FraudEngine.blend_params([w[n] for n in names], [S.CONF_MULT[n] for n in names])
    engine.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        for a, b in [(0, 7000), (7000, 20000)]:
            part = _slice(tx, a, b)
            n = b - a
            dev = {f: torch.from_numpy(np.ascontiguousarray(part[f])).cuda() for f in TXN_FIELDS}
            vec = torch.empty((n, 64), dtype=torch.float32, device="cuda")
            mp = torch.empty((2, n), dtype=torch.float64, device="cuda")
            fp = torch.empty(n, dtype=torch.float64, device="cuda")
            conf = torch.empty(n, dtype=torch.float64, device="cuda")
            dec = torch.empty(n, dtype=torch.uint8, device="cuda")
            risk = torch.empty(n, dtype=torch.uint8, device="cuda")
            engine.score_batch_device(params, [0, 1], {f: t.data_ptr() for f, t in dev.items()}, n, fp.data_ptr(),
                                      conf.data_ptr(), dec.data_ptr(), risk.data_ptr(), vec_ptr=vec.data_ptr(),
                                      model_probs_ptr=mp.data_ptr())
            torch.cuda.synchronize()
            _, rvec = orc.run(part)
            V = vec.cpu().numpy()
            _check_vectors(V, rvec)
            px, _, _ = oracle.xgb_predict(xgb, V)
            pi, _, _ = oracle.iforest_predict(ifm, V)
            M = mp.cpu().numpy()
            assert np.abs(M[0] - px).max() <= 1e-5 and np.abs(M[1] - pi).max() <= 1e-5
            FP, CF, DC, RK = fp.cpu().numpy(), conf.cpu().numpy(), dec.cpu().numpy(), risk.cpu().numpy()
            for i in range(0, n, 7):
                rfp, rcf, rdc, rrk = S.blend_row(names, [float(M[0, i]), float(M[1, i])], w)
                assert FP[i] == rfp and CF[i] == rcf
                assert DECISIONS[DC[i]] == rdc and RISK_LEVELS[RK[i]] == rrk
    finally:
        engine.set_stream(None)
