"""GPU parity at the BASELINE configurations' own shapes (BASELINE.json configs), through the product entry point
fd_score_batch_device (features on HBM-resident card state -> XGBoost + IsolationForest -> blend), against the
CPU oracle chain (oracle/oracle_features.c -> oracle_forest.c -> scoring_ref):

* config 3 at its stated size: 10 M cards (sliding windows, K = 16), XGBoost 500 x depth 8 + IsolationForest
  100, three 64 k micro-batches (the fused ensemble kernel's path);
* config 1's shape: the reference simulator's 100 k-transaction stream (10 k users, 5 k merchants) in
  micro-batches, state carried across them.

Bars: scoring vectors exact except the log slot (<= 1 f32 ulp, Java Math.log), model probabilities within the
north-star 1e-5 of the oracle forests on the same vectors, blend / decision / risk exact."""
import numpy as np
import pytest

from fdengine import FraudEngine, iforest_from_sklearn, synth, xgboost_from_json_doc
from fdengine._native import DECISIONS, RISK_LEVELS, TXN_FIELDS

pytestmark = pytest.mark.gpu


def _check_vectors(vec, rvec):
    same = vec == rvec
    if not same.all():
        bad = np.argwhere(~same)
        assert set(bad[:, 1].tolist()) <= {1}, f"non-transcendental slots differ: {sorted(set(bad[:, 1].tolist()))}"
        ulps = np.abs(vec.view(np.int32)[~same].astype(np.int64) - rvec.view(np.int32)[~same].astype(np.int64))
        assert ulps.max() <= 1


def _models(Xref, trees=500):
    xgb = xgboost_from_json_doc(synth.xgboost_doc(trees, 8, 64, Xref, seed=13))
    ifm = iforest_from_sklearn(synth.isolation_forest(Xref.astype(np.float64), n_estimators=100))
    return xgb, ifm


def _score_and_check(eng, orc, xgb, ifm, part, n):
    import torch

    import oracle
    from oracle import scoring_ref as S
    names = ["xgboost_primary", "isolation_forest"]
    w = S.normalized_weights({"xgboost_primary": 0.4, "isolation_forest": 0.05})
    params = FraudEngine.blend_params([w[k] for k in names], [S.CONF_MULT[k] for k in names])
    dev = {f: torch.from_numpy(np.ascontiguousarray(part[f])).cuda() for f in TXN_FIELDS}
    vec = torch.empty((n, 64), dtype=torch.float32, device="cuda")
    mp = torch.empty((2, n), dtype=torch.float64, device="cuda")
    outs = [torch.empty(n, dtype=t, device="cuda") for t in (torch.float64, torch.float64, torch.uint8, torch.uint8)]
    eng.score_batch_device(params, [0, 1], {f: t.data_ptr() for f, t in dev.items()}, n,
                           *[o.data_ptr() for o in outs], vec_ptr=vec.data_ptr(), model_probs_ptr=mp.data_ptr())
    torch.cuda.synchronize()
    _, rvec = orc.run(part)
    V = vec.cpu().numpy()
    _check_vectors(V, rvec)
    px, _, _ = oracle.xgb_predict(xgb, V)
    pi, _, _ = oracle.iforest_predict(ifm, V)
    M = mp.cpu().numpy()
    assert np.abs(M[0] - px).max() <= 1e-5 and np.abs(M[1] - pi).max() <= 1e-5
    fp, conf, dec, risk = oracle.blend_weighted(np.stack([M[0], M[1]]), [w[k] for k in names],
                                                [S.CONF_MULT[k] for k in names])
    FP, CF, DC, RK = (o.cpu().numpy() for o in outs)
    np.testing.assert_array_equal(FP, fp)
    np.testing.assert_array_equal(CF, conf)
    np.testing.assert_array_equal(DC, dec)
    np.testing.assert_array_equal(RK, risk)
    for i in range(0, n, 997):  # and the reference's own per-row blend (ensemble_predictor.py:252-369)
        rfp, _, rdc, rrk = S.blend_row(names, [float(M[0, i]), float(M[1, i])], w)
        assert FP[i] == rfp and DECISIONS[DC[i]] == rdc and RISK_LEVELS[RK[i]] == rrk
    return FP


@pytest.mark.timeout(900)
def test_config3_full_size():
    """10 M cards, 500 x 8 + 100 trees, 64 k micro-batches (BASELINE configs[2])."""
    from oracle.features_c import OracleFeatureState
    cards, B, K = 10_000_000, 65536, 16
    merch = synth.merchants_table(5000, seed=100)
    own = synth.owned_cards(cards, 0, 1, seed=42)
    cap = 1
    while cap < int(cards * 1.6) + 65536:
        cap *= 2
    tx = synth.txn_stream_cards(cards, merch, 4 * B, seed=200, card_seed=42, rate_per_s=2000.0)
    eng = FraudEngine(0)
    try:
        eng.state_init(cap, 1, K)
        eng.load_users(own["key"], own["avg_amount"], own["account_age_days"], own["device_fp"])
        eng.load_merchants(merch["fraud_rate"], merch["risk_multiplier"])
        orc = OracleFeatureState(cap, 1, K)
        orc.load_users(own["key"], own["avg_amount"], own["account_age_days"], own["device_fp"])
        orc.load_merchants(merch["fraud_rate"], merch["risk_multiplier"])
        # models on realistic vectors: the first micro-batch's features (engine; checked against the oracle)
        first = {k: v[:B] for k, v in tx.items()}
        V0 = eng.features(first)
        _, r0 = orc.run(first)
        _check_vectors(V0, r0)
        xgb, ifm = _models(V0[:8192])
        eng.load_forest(0, xgb)
        eng.load_forest(1, ifm)
        assert eng.state_info()["cards"] >= cards
        fps = [_score_and_check(eng, orc, xgb, ifm, {k: v[b * B:(b + 1) * B] for k, v in tx.items()}, B)
               for b in range(1, 4)]
        assert all(np.isfinite(f).all() for f in fps)
    finally:
        eng.close()


@pytest.mark.timeout(600)
def test_config1_simulator_stream(engine):
    """The reference simulator's 100 k transactions (10 k users, 5 k merchants; simulator.py:481-482) through
    the fused path in micro-batches, the card state carried across them (BASELINE configs[0])."""
    from oracle.features_c import OracleFeatureState
    pop = synth.population(10000, 5000, seed=1)
    tx = synth.txn_stream(pop, 100_000, seed=2)
    U, M = pop["users"], pop["merchants"]
    engine.state_init(1 << 15, 1, 16)
    engine.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    engine.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    orc = OracleFeatureState(1 << 15, 1, 16)
    orc.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    orc.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    warm = OracleFeatureState(1 << 15, 1, 16)
    warm.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
    warm.load_merchants(M["fraud_rate"], M["risk_multiplier"])
    _, Xref = warm.run({k: v[:20000] for k, v in tx.items()})
    xgb, ifm = _models(Xref[-8192:])
    engine.load_forest(0, xgb)
    engine.load_forest(1, ifm)
    cuts = [0, 1000, 33768, 66536, 100_000]  # a latency-size batch, then 32 k + 32 k (fused) + the rest
    for a, b in zip(cuts[:-1], cuts[1:]):
        _score_and_check(engine, orc, xgb, ifm, {k: v[a:b] for k, v in tx.items()}, b - a)
