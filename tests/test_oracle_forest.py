"""CPU: pin the forest oracle, and prove the engine's repacked layout equivalent to the original
trees (walked in Python exactly as the HIP kernel walks it) — no GPU needed.

XGBoost parity against the library itself is UNPINNED (xgboost==2.0.3 is not installable offline);
these known-answer trees pin the restated semantics: `x < split_condition` goes left (ties right),
NaN follows default_left, f32 leaf weights summed in tree order from ProbToMargin(base_score),
p = 1/(1+exp(-margin)) in f32.
"""
import json

import numpy as np
import pytest

import oracle
from oracle import forest_ref
from conftest import GOLDEN
from fdengine import ForestArrays, iforest_from_sklearn, pack_forest_host, synth, xgboost_from_json_doc
from fdengine import _native as N


def _stump_doc(thr, lw, rw, dl, base_score="5E-1"):
    return {"learner": {
        "gradient_booster": {"name": "gbtree", "model": {"trees": [{
            "left_children": [1, -1, -1], "right_children": [2, -1, -1], "split_indices": [0, 0, 0],
            "split_conditions": [thr, lw, rw], "default_left": [dl, 0, 0], "split_type": [0, 0, 0],
            "tree_param": {"num_feature": "2", "num_nodes": "3", "size_leaf_vector": "1"}}]}},
        "learner_model_param": {"base_score": base_score, "num_class": "0", "num_feature": "2"},
        "objective": {"name": "binary:logistic"}}}


def test_xgb_known_answers():
    fa = xgboost_from_json_doc(_stump_doc(0.5, -1.25, 2.0, 1))
    X = np.array([[0.25, 0], [0.5, 0], [0.75, 0], [np.nan, 0]], np.float32)
    prob, margin, leaf = oracle.xgb_predict(fa, X, want_leaf=True)
    # x < 0.5 -> left (-1.25); x == 0.5 -> right (2.0); NaN -> default_left
    np.testing.assert_array_equal(margin, np.float32([-1.25, 2.0, 2.0, -1.25]))
    np.testing.assert_array_equal(leaf[:, 0], [1, 2, 2, 1])
    expect = (1.0 / (1.0 + np.exp(-np.float64(margin)))).astype(np.float32)
    assert np.abs(prob - expect).max() <= 1e-7
    # base_score 0.2 -> margin seed logit(0.2) = -ln 4
    fa2 = xgboost_from_json_doc(_stump_doc(0.5, 0.0, 0.0, 0, base_score="2E-1"))
    _, m2, _ = oracle.xgb_predict(fa2, X[:1])
    assert abs(float(m2[0]) - (-np.log(4.0))) < 1e-6


def test_xgb_loader_rejects_unsupported():
    from fdengine import UnsupportedModel
    d = _stump_doc(0.5, 0, 0, 0)
    d["learner"]["objective"]["name"] = "reg:squarederror"
    with pytest.raises(UnsupportedModel):
        xgboost_from_json_doc(d)
    d = _stump_doc(0.5, 0, 0, 0)
    d["learner"]["gradient_booster"]["model"]["trees"][0]["split_type"] = [1, 0, 0]
    with pytest.raises(UnsupportedModel):
        xgboost_from_json_doc(d)


def test_xgb_c_oracle_matches_python_walker_and_packed_layout():
    X = synth.feature_matrix(300, 30, seed=3, nan_frac=0.05)
    fa = xgboost_from_json_doc(synth.xgboost_doc(25, 8, 30, X, seed=4, p_leaf=0.2, base_score=0.3))
    _, margin, leaf = oracle.xgb_predict(fa, X, want_leaf=True)
    blob, ids, info = pack_forest_host(fa)
    assert info.depth == 8 and info.chunk in (4, 8, 12, 16)
    for r in range(0, 300, 7):
        m, lv = forest_ref.xgb_walk(fa, X[r])
        pm, pl = forest_ref.packed_walk(blob, ids, info, True, X[r])
        assert np.float32(m) == margin[r] == np.float32(pm)
        assert lv == list(leaf[r]) == pl


def test_iforest_oracle_pinned_by_sklearn():
    Xtr = synth.feature_matrix(1500, 16, seed=8).astype(np.float64)
    m = synth.isolation_forest(Xtr, n_estimators=30)
    fa = iforest_from_sklearn(m)
    X = synth.feature_matrix(400, 16, seed=9)
    prob, depth, leaf = oracle.iforest_predict(fa, X, want_leaf=True)
    np.testing.assert_array_equal(leaf, np.stack([e.apply(X) for e in m.estimators_], 1))
    ref = 1.0 / (1.0 + np.exp(m.decision_function(X)))
    assert np.abs(prob - ref).max() <= 1e-12
    blob, ids, info = pack_forest_host(fa)
    for r in range(0, 400, 13):
        d, lv = forest_ref.iforest_walk(fa, X[r])
        pd_, pl = forest_ref.packed_walk(blob, ids, info, False, X[r])
        assert d == depth[r] == pd_
        assert lv == list(leaf[r]) == pl


def test_sklearn_threshold_rewrite_is_exact_at_the_boundary():
    """sklearn's (double)x <= thr_f64 must equal the engine's x < t_f32 for every f32 x near thr."""
    rng = np.random.default_rng(0)
    left = np.array([1, -1, -1]); right = np.array([2, -1, -1])
    for _ in range(200):
        thr = float(rng.normal() * 10.0 ** int(rng.integers(-3, 4)))
        fa = ForestArrays(kind=N.FD_FOREST_SKLEARN_IFOREST, num_feature=1, offsets=np.array([0, 3]), left=left,
                          right=right, feature=np.zeros(3, int), threshold=np.array([thr, 0, 0]),
                          default_left=np.zeros(3, int), leaf_value=np.array([0, 1.0, 2.0]), if_denominator=1.0)
        blob, ids, info = pack_forest_host(fa)
        f = np.float32(thr)
        xs = [np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))]
        for x in xs:
            d, _ = forest_ref.iforest_walk(fa, [x])
            pd_, _ = forest_ref.packed_walk(blob, ids, info, False, [x])
            assert d == pd_, (thr, x)


# ---------------------------------------------------------------- binned layout (forest_kernel4)

from fdengine.engine import pack_forest_binned_host  # noqa: E402


@pytest.mark.parametrize("max_bin", [256, None])
def test_binned_layout_matches_oracle_xgb(max_bin):
    X = synth.feature_matrix(300, 30, seed=3, nan_frac=0.05)
    fa = xgboost_from_json_doc(synth.xgboost_doc(25, 8, 30, X, seed=4, p_leaf=0.2, base_score=0.3, max_bin=max_bin))
    _, margin, leaf = oracle.xgb_predict(fa, X, want_leaf=True)
    blob, ids, info = pack_forest_host(fa)
    bblob, thr, off, binfo = pack_forest_binned_host(fa)
    assert binfo.layout == 1 and binfo.depth == 8 and binfo.tree_bytes == 256 * 4 + 256 * 4
    assert len(off) == 31 and off[0] == 0 and off[-1] == len(thr) == binfo.n_thresholds
    for f in range(30):
        t = thr[off[f]:off[f + 1]]
        assert np.all(np.diff(t) > 0)  # ascending, distinct
    if max_bin:
        assert np.diff(off).max() <= 255
    assert binfo.bin_steps == (1 << int(np.floor(np.log2(np.diff(off).max()))))
    for r in range(0, 300, 7):
        pm, pl = forest_ref.packed_walk_binned(bblob, ids, thr, off, binfo, True, X[r])
        assert np.float32(pm) == margin[r]
        assert pl == list(leaf[r])


def test_binned_layout_matches_sklearn_iforest():
    Xtr = synth.feature_matrix(1500, 16, seed=8).astype(np.float64)
    m = synth.isolation_forest(Xtr, n_estimators=30)
    fa = iforest_from_sklearn(m)
    X = synth.feature_matrix(200, 16, seed=9, nan_frac=0.02)
    prob, depth, leaf = oracle.iforest_predict(fa, X, want_leaf=True)
    bblob, thr, off, binfo = pack_forest_binned_host(fa)
    _, ids, _ = pack_forest_host(fa)
    for r in range(0, 200, 9):
        d, lv = forest_ref.packed_walk_binned(bblob, ids, thr, off, binfo, False, X[r])
        assert d == depth[r]
        assert lv == list(leaf[r])


def test_binned_sklearn_threshold_boundary():
    rng = np.random.default_rng(1)
    left = np.array([1, -1, -1]); right = np.array([2, -1, -1])
    for _ in range(100):
        thr = float(rng.normal() * 10.0 ** int(rng.integers(-3, 4)))
        fa = ForestArrays(kind=N.FD_FOREST_SKLEARN_IFOREST, num_feature=1, offsets=np.array([0, 3]), left=left,
                          right=right, feature=np.zeros(3, int), threshold=np.array([thr, 0, 0]),
                          default_left=np.zeros(3, int), leaf_value=np.array([0, 1.0, 2.0]), if_denominator=1.0)
        bblob, thr_t, off, binfo = pack_forest_binned_host(fa)
        _, ids, _ = pack_forest_host(fa)
        f = np.float32(thr)
        for x in (np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))):
            d, _ = forest_ref.iforest_walk(fa, [x])
            bd, _ = forest_ref.packed_walk_binned(bblob, ids, thr_t, off, binfo, False, [x])
            assert d == bd, (thr, x)


def test_binned_layout_refused_beyond_65534_thresholds():
    X = np.random.default_rng(2).normal(size=(200000, 1)).astype(np.float32)
    fa = xgboost_from_json_doc(synth.xgboost_doc(400, 8, 1, X, seed=5, max_bin=None))
    with pytest.raises(N.NativeError) as ei:
        pack_forest_binned_host(fa)
    assert ei.value.code == N.FD_ERR_UNSUPPORTED
    blob, ids, info = pack_forest_host(fa)  # the threshold layout still packs
    assert info.layout == 0 and info.n_thresholds == 0
