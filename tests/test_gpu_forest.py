"""GPU parity: the HIP forest kernel (through the C-ABI) against the CPU oracle on the same seeded
inputs. Bars (BASELINE.json north_star): leaf indices bit-exact; probabilities within 1e-5 absolute.
This suite also holds the engine to more than that bar: XGBoost margins are the same f32 sum sequence
(bit-exact) and IsolationForest path-length sums the same f64 sequence (bit-exact)."""
import numpy as np
import pytest

import oracle
from fdengine import FraudEngine, iforest_from_sklearn, synth, xgboost_from_json_doc
from fdengine import _native as N

pytestmark = pytest.mark.gpu

PROB_TOL = 1e-5  # north_star: fraud probabilities within 1e-5 absolute


def _xgb_case(engine, slot, n, n_trees, depth, nf, seed, p_leaf=0.0, nan_frac=0.0, ld=None, base_score=0.5,
              max_bin=256):
    X = synth.feature_matrix(n, nf, seed=seed, nan_frac=nan_frac)
    doc = synth.xgboost_doc(n_trees, depth, nf, synth.feature_matrix(512, nf, seed=seed + 1), seed=seed + 2,
                            p_leaf=p_leaf, base_score=base_score, max_bin=max_bin)
    fa = xgboost_from_json_doc(doc)
    if ld is not None and ld < nf:
        X = np.ascontiguousarray(X[:, :ld])
    engine.load_forest(slot, fa)
    prob, raw, leaf = engine.predict(slot, X, want_raw=True, want_leaf=True)
    rp, rm, rl = oracle.xgb_predict(fa, X, want_leaf=True)
    return prob, raw, leaf, rp, rm, rl


@pytest.mark.parametrize("n", [1, 255, 256, 257, 4099])
def test_xgb_parity_sizes(engine, n):
    prob, raw, leaf, rp, rm, rl = _xgb_case(engine, 0, n, 64, 8, 50, seed=11)
    np.testing.assert_array_equal(leaf, rl)
    np.testing.assert_array_equal(raw.astype(np.float32), rm)  # same f32 sequence
    assert np.abs(prob - rp.astype(np.float64)).max() <= PROB_TOL


@pytest.mark.parametrize("depth", [1, 2, 5, 8, 9, 10])
def test_xgb_parity_depths(engine, depth):
    prob, raw, leaf, rp, rm, rl = _xgb_case(engine, 1, 1000, 37, depth, 20, seed=20 + depth, p_leaf=0.2)
    np.testing.assert_array_equal(leaf, rl)
    np.testing.assert_array_equal(raw.astype(np.float32), rm)
    assert np.abs(prob - rp).max() <= PROB_TOL


def test_xgb_missing_values_and_short_rows(engine):
    # NaN -> default_left; columns beyond the caller's ld are missing (DMatrix semantics)
    prob, raw, leaf, rp, rm, rl = _xgb_case(engine, 2, 3000, 100, 8, 50, seed=31, p_leaf=0.1, nan_frac=0.1)
    np.testing.assert_array_equal(leaf, rl)
    np.testing.assert_array_equal(raw.astype(np.float32), rm)
    prob, raw, leaf, rp, rm, rl = _xgb_case(engine, 2, 700, 50, 7, 50, seed=32, ld=33)
    np.testing.assert_array_equal(leaf, rl)
    np.testing.assert_array_equal(raw.astype(np.float32), rm)
    assert np.abs(prob - rp).max() <= PROB_TOL


def test_xgb_base_score(engine):
    prob, raw, leaf, rp, rm, rl = _xgb_case(engine, 3, 500, 20, 6, 16, seed=41, base_score=0.137)
    np.testing.assert_array_equal(raw.astype(np.float32), rm)
    assert np.abs(prob - rp).max() <= PROB_TOL


def test_xgb_config2_full_batch(engine):
    """BASELINE config 2 at full size: 500 trees x depth 8, 50 features, 64k micro-batch."""
    prob, raw, leaf, rp, rm, rl = _xgb_case(engine, 4, 65536, 500, 8, 50, seed=51)
    np.testing.assert_array_equal(leaf, rl)
    np.testing.assert_array_equal(raw.astype(np.float32), rm)
    assert np.abs(prob - rp).max() <= PROB_TOL


def test_xgb_config2_timed_kernel(engine):
    """the kernel config 2's bench line times — fd_forest_predict with no leaf ids at 500 trees x
    depth 8, 50 features, 64 k rows selects the fused single-forest ensemble_kernel<8,2> (engine counter
    ensemble_single_launches proves it ran, twice) — against oracle.xgb_predict: probabilities within 1e-5 on the
    probability-only launch (the bench's exact call), and the same kernel's f32 margins bit-identical when its raw
    output is requested (model_manager.py:309-311)."""
    X = synth.feature_matrix(65536, 50, seed=71, nan_frac=0.01)
    doc = synth.xgboost_doc(500, 8, 50, synth.feature_matrix(512, 50, seed=72), seed=73, p_leaf=0.05)
    fa = xgboost_from_json_doc(doc)
    engine.load_forest(6, fa)
    c0 = engine.counter("ensemble_single_launches")
    prob = engine.predict(6, X)  # probabilities only: the bench's timed call
    assert engine.counter("ensemble_single_launches") - c0 == 1
    prob2, raw = engine.predict(6, X, want_raw=True)  # the same kernel with its raw-score output
    assert engine.counter("ensemble_single_launches") - c0 == 2
    rp, rm, _ = oracle.xgb_predict(fa, X)
    assert np.abs(prob - rp).max() <= PROB_TOL
    np.testing.assert_array_equal(prob2, prob)
    np.testing.assert_array_equal(raw.astype(np.float32), rm)  # the reference's f32 sum sequence, bit for bit
    np.testing.assert_array_equal(raw, raw.astype(np.float32).astype(np.float64))


def test_iforest_parity_vs_sklearn(engine):
    Xtr = synth.feature_matrix(4000, 64, seed=61).astype(np.float64)
    m = synth.isolation_forest(Xtr)
    fa = iforest_from_sklearn(m)
    X = synth.feature_matrix(5000, 64, seed=62)
    X[::97, 3] = np.nan  # missing_go_to_left path
    engine.load_forest(5, fa)
    prob, raw, leaf = engine.predict(5, X, want_raw=True, want_leaf=True)
    rp, rd, rl = oracle.iforest_predict(fa, X, want_leaf=True)
    np.testing.assert_array_equal(leaf, rl)
    np.testing.assert_array_equal(raw, rd)  # same f64 sequence
    assert np.abs(prob - rp).max() <= PROB_TOL
    # and against sklearn + the reference's transform itself (finite rows)
    Xf = synth.feature_matrix(2000, 64, seed=63)
    p2 = engine.predict(5, Xf)
    ref = 1.0 / (1.0 + np.exp(m.decision_function(Xf)))
    assert np.abs(p2 - ref).max() <= 1e-12
    np.testing.assert_array_equal(engine.predict(5, Xf, want_leaf=True)[1],
                                  np.stack([e.apply(Xf) for e in m.estimators_], 1))


def test_empty_batch_and_unloaded_slot(engine):
    engine.load_forest(6, xgboost_from_json_doc(synth.xgboost_doc(3, 3, 4, synth.feature_matrix(64, 4))))
    out = engine.predict(6, np.zeros((0, 4), np.float32))
    assert out.shape == (0,)
    with pytest.raises(ValueError):
        engine.predict(7, np.zeros((3, 4), np.float32))


def test_device_pointer_path_matches_host_path(engine):
    import torch
    X = synth.feature_matrix(3000, 50, seed=71)
    fa = xgboost_from_json_doc(synth.xgboost_doc(80, 8, 50, X, seed=72))
    engine.load_forest(0, fa)
    host = engine.predict(0, X)
    dX = torch.from_numpy(X).cuda()
    dp = torch.empty(3000, dtype=torch.float64, device="cuda")
    engine.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        engine.predict_device(0, dX.data_ptr(), 3000, 50, dp.data_ptr())
        torch.cuda.synchronize()
    finally:
        engine.set_stream(None)
    np.testing.assert_array_equal(dp.cpu().numpy(), host)


@pytest.mark.parametrize("depth", [1, 2, 3, 4, 6, 8])
@pytest.mark.parametrize("variant", [3, 8])
def test_kernel4_depths(engine, depth, variant):
    """The binned 1024-thread kernel (option 3) and its node-only-chunk form with leaves from global memory
    (option 8, kernel 6) across depths, ragged trees, NaNs, odd tree counts."""
    engine.set_option("forest_kernel", variant)
    try:
        prob, raw, leaf, rp, rm, rl = _xgb_case(engine, 1, 777, 45, depth, 21, seed=190 + depth, p_leaf=0.2,
                                                nan_frac=0.02)
        np.testing.assert_array_equal(leaf, rl)
        np.testing.assert_array_equal(raw.astype(np.float32), rm)
        assert np.abs(prob - rp).max() <= PROB_TOL
    finally:
        engine.set_option("forest_kernel", 0)


@pytest.mark.parametrize("max_bin", [256, None])
@pytest.mark.parametrize("variant", [1, 2, 3, 6, 8])
def test_kernel_variants_agree(engine, variant, max_bin):
    """Every forest kernel (256-thread; 1024-thread tree-split on the threshold layout; 1024-thread on
    the binned layout) gives the oracle's bits, for hist-style and raw-valued split thresholds."""
    engine.set_option("forest_kernel", variant)
    try:
        prob, raw, leaf, rp, rm, rl = _xgb_case(engine, 0, 3001, 203, 8, 50, seed=81, p_leaf=0.05, nan_frac=0.01,
                                                max_bin=max_bin)
        np.testing.assert_array_equal(leaf, rl)
        np.testing.assert_array_equal(raw.astype(np.float32), rm)
        assert np.abs(prob - rp).max() <= PROB_TOL
        Xtr = synth.feature_matrix(2000, 40, seed=82).astype(np.float64)
        fa = iforest_from_sklearn(synth.isolation_forest(Xtr, n_estimators=37))
        X = synth.feature_matrix(1500, 40, seed=83)
        engine.load_forest(1, fa)
        p, d, lf = engine.predict(1, X, want_raw=True, want_leaf=True)
        rp2, rd2, rl2 = oracle.iforest_predict(fa, X, want_leaf=True)
        np.testing.assert_array_equal(lf, rl2)
        np.testing.assert_array_equal(d, rd2)
    finally:
        engine.set_option("forest_kernel", 0)


def test_removed_kernel_options_refused(engine):
    """options measured slower and removed (kernel 5, walk4t, kernel 6's dynamic / skewed schedules) are refused"""
    for v in (4, 5, 7, 9, 10):
        with pytest.raises(N.NativeError):
            engine.set_option("forest_kernel", v)


def test_unbinnable_forest_falls_back(engine):
    """> 65534 distinct thresholds in a feature: auto picks the threshold-layout kernel (still exact);
    forcing the binned kernel is refused."""
    Xr = np.random.default_rng(2).normal(size=(200000, 1)).astype(np.float32)
    fa = xgboost_from_json_doc(synth.xgboost_doc(400, 8, 1, Xr, seed=5, max_bin=None))
    engine.load_forest(0, fa)
    X = synth.feature_matrix(1000, 1, seed=6, nan_frac=0.05)
    prob, raw, leaf = engine.predict(0, X, want_raw=True, want_leaf=True)
    rp, rm, rl = oracle.xgb_predict(fa, X, want_leaf=True)
    np.testing.assert_array_equal(leaf, rl)
    np.testing.assert_array_equal(raw.astype(np.float32), rm)
    engine.set_option("forest_kernel", 3)
    try:
        with pytest.raises(N.NativeError):
            engine.predict(0, X)
    finally:
        engine.set_option("forest_kernel", 0)
