"""CPU: the engine's C++ reader of the reference's XGBoost JSON model file (fd_xgboost_json_read, the
host half of fd_load_xgboost_json) flattens a file exactly as the Python reader (fdengine/forest.py,
pinned to the XGBoost 2.0.3 schema) and rejects what it rejects."""
import json

import numpy as np
import pytest

from fdengine import _native as N
from fdengine import synth
from fdengine.engine import read_xgboost_json_native
from fdengine.forest import load_xgboost_json


@pytest.mark.parametrize("depth,p_leaf,base", [(8, 0.0, 0.5), (6, 0.2, 0.137), (1, 0.0, 0.9)])
def test_native_reader_equals_python_reader(tmp_path, depth, p_leaf, base):
    X = synth.feature_matrix(1024, 33, seed=depth)
    path = tmp_path / "fraud_classifier.json"
    synth.write_xgboost_json(str(path), synth.xgboost_doc(37, depth, 33, X, seed=3, p_leaf=p_leaf, base_score=base,
                                                          max_bin=None))
    a, b = read_xgboost_json_native(path), load_xgboost_json(str(path))
    assert a.num_feature == b.num_feature and a.base_score == b.base_score and a.n_trees == b.n_trees
    for k in ("offsets", "left", "right", "feature", "threshold", "default_left", "leaf_value"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)


def test_native_reader_rejects_like_the_reference(tmp_path):
    X = synth.feature_matrix(256, 4, seed=1)
    doc = synth.xgboost_doc(3, 3, 4, X, seed=2)
    bad = json.loads(json.dumps(doc))
    bad["learner"]["objective"]["name"] = "reg:squarederror"
    p = tmp_path / "m.json"
    p.write_text(json.dumps(bad))
    with pytest.raises(N.NativeError) as ei:
        read_xgboost_json_native(p)
    assert ei.value.code == N.FD_ERR_UNSUPPORTED
    cat = json.loads(json.dumps(doc))
    cat["learner"]["gradient_booster"]["model"]["trees"][0]["split_type"][0] = 1
    p.write_text(json.dumps(cat))
    with pytest.raises(N.NativeError) as ei:
        read_xgboost_json_native(p)
    assert ei.value.code == N.FD_ERR_UNSUPPORTED
    p.write_text(json.dumps(doc)[:-40])  # truncated file
    with pytest.raises(N.NativeError) as ei:
        read_xgboost_json_native(p)
    assert ei.value.code == N.FD_ERR_INVALID_ARG
    with pytest.raises(N.NativeError) as ei:
        read_xgboost_json_native(tmp_path / "missing.json")
    assert ei.value.code == N.FD_ERR_IO
