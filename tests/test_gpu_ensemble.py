"""GPU parity of the fused ensemble kernel (csrc/ensemble.hip): XGBoost + IsolationForest walked over one
binned tile (merged threshold tables) with the blend epilogue, used for large batches (>= 128 tiles of 256)
when the present models are one XGBoost and one IsolationForest.

Bars: probabilities within 1e-5 of the oracle chain (north star), and — stronger — every output bit-identical
to the per-model path (one forest kernel per model + blend kernel, engine option ensemble = 0),
because the walk reproduces the reference's sequential f32 margin / f64 path-length sums exactly. Covers the
binning plans (tables staged in one pass, several passes, a table too large for LDS searched in global
memory), depth padding (XGBoost depth 6 with an IsolationForest of depth 8), NaNs and short rows, reversed
model order, all three blend strategies, and the routed-records output."""
import numpy as np
import pytest

import oracle
from fdengine import FraudEngine, iforest_from_sklearn, synth, xgboost_from_json_doc
from fdengine._native import FD_TIMING_ENSEMBLE, NativeError
from oracle import scoring_ref as S

pytestmark = pytest.mark.gpu

N = 40000  # 157 tiles: the fused path


def _models(nf, depth_x, n_trees=120, max_bin=256, seed=1, n_if=60, ref_rows=4096):
    Xr = synth.feature_matrix(ref_rows, nf, seed=seed)
    xgb = xgboost_from_json_doc(synth.xgboost_doc(n_trees, depth_x, nf, Xr, seed=seed + 1, p_leaf=0.1,
                                                  max_bin=max_bin, base_score=0.3))
    ifm = iforest_from_sklearn(synth.isolation_forest(Xr.astype(np.float64), n_estimators=n_if))
    return xgb, ifm


def _score(engine, params, slots, X, fused):
    engine.set_option("ensemble", 1 if fused else 0)
    try:
        engine.read_timing()
        engine.set_timing(True)
        out = engine.score_matrix(params, slots, X)
        engine.set_timing(False)
        used = engine.read_timing(FD_TIMING_ENSEMBLE)[1] > 0
    finally:
        engine.set_option("ensemble", 1)
    return out, used


def _check(engine, xgb, ifm, X, names=("xgboost_primary", "isolation_forest"), strategy=0):
    engine.load_forest(0, xgb)
    engine.load_forest(1, ifm)
    slot_of = {"xgboost_primary": 0, "isolation_forest": 1}
    slots = [slot_of[n] for n in names]
    w = S.normalized_weights({"xgboost_primary": 0.4, "isolation_forest": 0.05})
    params = FraudEngine.blend_params([w[n] for n in names], [S.CONF_MULT[n] for n in names], strategy=strategy)
    fused, used = _score(engine, params, slots, X, True)
    assert used, "the fused ensemble kernel did not run"
    per_model, used2 = _score(engine, params, slots, X, False)
    assert not used2
    for a, b in zip(fused, per_model):  # model probs, fp, conf, decision, risk: identical bits
        np.testing.assert_array_equal(a, b)
    px, _, _ = oracle.xgb_predict(xgb, X)
    pi, _, _ = oracle.iforest_predict(ifm, X)
    ref = {"xgboost_primary": px.astype(np.float64), "isolation_forest": pi}
    mp = fused[0]
    for m, n in enumerate(names):
        assert np.abs(mp[m] - ref[n]).max() <= 1e-5
    strat = ("weighted_average", "voting", "stacking")[strategy]
    fp = fused[1]
    for i in range(0, len(X), 97):
        rfp, rcf, _, _ = S.blend_row(list(names), [float(mp[0, i]), float(mp[1, i])], w, strat)
        assert fp[i] == rfp and fused[2][i] == rcf


@pytest.mark.parametrize("chunks", [1, 2])
@pytest.mark.parametrize("strategy", [0, 1, 2])
def test_fused_matches_per_model_and_oracle(engine, strategy, chunks):
    """both chunk layouts (engine option ensemble_chunks: 1 wide 24 / 16 trees, 2 compact 20 / 12)"""
    xgb, ifm = _models(64, 8, seed=3)
    X = synth.feature_matrix(N, 64, seed=4, nan_frac=0.01)
    engine.set_option("ensemble_chunks", chunks)
    try:
        _check(engine, xgb, ifm, X, strategy=strategy)
    finally:
        engine.set_option("ensemble_chunks", 0)


def test_reversed_model_order_and_depth_padding(engine):
    xgb, ifm = _models(40, 6, n_trees=90, seed=5)  # XGBoost depth 6 padded to the IsolationForest's 8
    X = synth.feature_matrix(N + 123, 40, seed=6)
    _check(engine, xgb, ifm, X, names=("isolation_forest", "xgboost_primary"))


def test_shallow_forests(engine):
    """depth 3 and depth 2 forests (IsolationForest max_samples 8 / 4) through the fused kernel; one chunk of each
    forest only (17 + 5 trees) included"""
    for d, s, nx, ni in ((3, 31, 70, 20), (2, 33, 70, 20), (3, 35, 17, 5)):
        Xr = synth.feature_matrix(4096, 24, seed=s)
        xgb = xgboost_from_json_doc(synth.xgboost_doc(nx, d, 24, Xr, seed=s + 1, base_score=0.4))
        ifm = iforest_from_sklearn(synth.isolation_forest(Xr.astype(np.float64), n_estimators=ni, max_samples=2 ** d))
        X = synth.feature_matrix(N, 24, seed=s + 2, nan_frac=0.01)
        _check(engine, xgb, ifm, X)


def test_short_rows_are_missing_columns(engine):
    xgb, ifm = _models(64, 8, n_trees=50, seed=7)
    X = np.ascontiguousarray(synth.feature_matrix(N, 64, seed=8)[:, :48])  # ld 48 < 64: the rest NaN
    engine.load_forest(0, xgb)
    engine.load_forest(1, ifm)
    params = FraudEngine.blend_params([0.4 / 0.45, 0.05 / 0.45], [1.0, 0.5])
    fused, used = _score(engine, params, [0, 1], X, True)
    per_model, _ = _score(engine, params, [0, 1], X, False)
    assert used
    for a, b in zip(fused, per_model):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("chunks", [1, 2])
def test_multi_pass_and_global_binning(engine, chunks):
    """Raw-valued thresholds: thousands of distinct thresholds per feature, so the merged tables take several
    LDS passes (fewer staging bytes in the compact layout: more passes); one 2-feature model whose feature-0
    table alone exceeds the LDS space (global search)."""
    engine.set_option("ensemble_chunks", chunks)
    try:
        xgb, ifm = _models(64, 8, n_trees=400, max_bin=None, seed=9, ref_rows=20000)
        X = synth.feature_matrix(N, 64, seed=10, nan_frac=0.005)
        _check(engine, xgb, ifm, X)
        Xr = np.random.default_rng(11).normal(size=(60000, 2)).astype(np.float32)
        xgb2 = xgboost_from_json_doc(synth.xgboost_doc(300, 8, 2, Xr, seed=12, max_bin=None))
        ifm2 = iforest_from_sklearn(synth.isolation_forest(Xr[:8192].astype(np.float64), n_estimators=30))
        X2 = np.random.default_rng(13).normal(size=(N, 2)).astype(np.float32)
        _check(engine, xgb2, ifm2, X2)
    finally:
        engine.set_option("ensemble_chunks", 0)


def test_reload_invalidates_the_joint_repack(engine):
    xgb, ifm = _models(64, 8, n_trees=60, seed=14)
    X = synth.feature_matrix(N, 64, seed=15)
    _check(engine, xgb, ifm, X)
    xgb_b, _ = _models(64, 8, n_trees=70, seed=16)
    _check(engine, xgb_b, ifm, X)  # a different model in slot 0: the cached plan must not be reused


def test_sampled_kernel_timing(engine):
    """engine option "timing_every" = 3: HIP events on launches 0, 3, 6 of each kind; averages unchanged in kind"""
    xgb, ifm = _models(64, 8, n_trees=40, seed=17)
    engine.load_forest(0, xgb)
    engine.load_forest(1, ifm)
    X = synth.feature_matrix(N, 64, seed=18)
    params = FraudEngine.blend_params([0.4 / 0.45, 0.05 / 0.45], [1.0, 0.5])
    engine.read_timing()
    engine.set_option("timing_every", 3)
    try:
        engine.set_timing(True)
        outs = [engine.score_matrix(params, [0, 1], X) for _ in range(7)]
        engine.set_timing(False)
        ms, launches = engine.read_timing(FD_TIMING_ENSEMBLE)
    finally:
        engine.set_option("timing_every", 1)
    assert launches == 3 and ms > 0.0
    for o in outs[1:]:
        for u, v in zip(o, outs[0]):
            np.testing.assert_array_equal(u, v)
    with pytest.raises(NativeError):
        engine.set_option("timing_every", 0)


@pytest.mark.parametrize("kind,depth", [("xgb", 8), ("xgb", 6), ("if", 8)])
def test_single_forest_fused_equals_kernel6(engine, kind, depth):
    """fd_forest_predict on a large batch without raw / leaf outputs runs the fused kernel over the one forest
    (_predict_xgboost / _predict_sklearn, ml/models/model_manager.py:309-311, 338-346): probabilities
    bit-identical to forest kernel 6 (engine option ensemble = 0), NaNs and short rows included; and with raw
    margins requested the call keeps kernel 6."""
    nf = 64
    xgb, ifm = _models(nf, depth, n_trees=150, n_if=50, seed=11 + depth)
    model = xgb if kind == "xgb" else ifm
    engine.load_forest(2, model)
    X = synth.feature_matrix(N, nf, seed=5).astype(np.float32)
    X[::113, 7] = np.nan
    X[5::251, :] = np.nan
    fused = engine.predict(2, X)
    engine.set_option("ensemble", 0)
    try:
        k6, raw = engine.predict(2, X, want_raw=True)
        k6b = engine.predict(2, X)
    finally:
        engine.set_option("ensemble", 1)
    np.testing.assert_array_equal(fused, k6)
    np.testing.assert_array_equal(fused, k6b)
    _, raw1 = engine.predict(2, X, want_raw=True)  # raw requested: kernel 6 even with the option on
    np.testing.assert_array_equal(raw1, raw)
    short = np.ascontiguousarray(X[:, :48])  # rows shorter than num_feature: missing columns
    np.testing.assert_array_equal(engine.predict(2, short), _k6(engine, 2, short))
    ref = oracle.xgb_predict(model, X)[0].astype(np.float64) if kind == "xgb" else oracle.iforest_predict(model, X)[0]
    assert np.abs(fused - ref).max() <= 1e-5


def _k6(engine, slot, X):
    engine.set_option("ensemble", 0)
    try:
        return engine.predict(slot, X)
    finally:
        engine.set_option("ensemble", 1)


@pytest.mark.parametrize("n_trees", [1, 10, 30])
def test_single_forest_few_chunks(engine, n_trees):
    """one forest of one or two chunks through the fused kernel: probabilities bit-identical to forest kernel 6"""
    Xr = synth.feature_matrix(4096, 32, seed=41)
    xgb = xgboost_from_json_doc(synth.xgboost_doc(n_trees, 8, 32, Xr, seed=42, base_score=0.2))
    engine.load_forest(3, xgb)
    X = synth.feature_matrix(N, 32, seed=43, nan_frac=0.01)
    np.testing.assert_array_equal(engine.predict(3, X), _k6(engine, 3, X))
