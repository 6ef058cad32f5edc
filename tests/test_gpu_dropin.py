"""GPU: the drop-in host API (ModelManager / EnsemblePredictor mirrors) over real model FILES in the
reference's formats and directory layout, checked against the oracle chain
(oracle XGBoost + oracle IF + scoring_ref blend)."""
import asyncio
import json

import numpy as np
import pytest

import oracle
from conftest import GOLDEN
from oracle import features_ref as FR
from oracle import scoring_ref as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model_dir(tmp_path_factory):
    import joblib
    from fdengine import synth
    d = tmp_path_factory.mktemp("models")
    (d / "xgboost").mkdir()
    (d / "sklearn").mkdir()
    Xref = synth.feature_matrix(4096, 64, seed=3)
    synth.write_xgboost_json(str(d / "xgboost" / "fraud_classifier.json"),
                             synth.xgboost_doc(120, 8, 64, Xref, seed=4, p_leaf=0.1, base_score=0.2))
    joblib.dump(synth.isolation_forest(Xref.astype(np.float64)), d / "sklearn" / "isolation_forest.joblib")
    return d


def _stack(model_dir, strategy="weighted_average"):
    from fdengine.ensemble import EnsemblePredictor
    from fdengine.model_manager import ModelManager
    from fdengine.registry import ScoringConfig
    cfg = ScoringConfig(str(model_dir))
    cfg.disable_model("bert_text")
    cfg.disable_model("graph_neural")
    cfg.ensemble.strategy = strategy
    mm = ModelManager(cfg, device=0)
    asyncio.run(mm.load_all_models())
    return cfg, mm, EnsemblePredictor(mm, cfg)


def _oracle_models(model_dir):
    import joblib
    from fdengine import iforest_from_sklearn, load_xgboost_json
    return (load_xgboost_json(str(model_dir / "xgboost" / "fraud_classifier.json")),
            iforest_from_sklearn(joblib.load(model_dir / "sklearn" / "isolation_forest.joblib")))


@pytest.mark.parametrize("strategy", ["weighted_average", "voting", "stacking"])
def test_predict_and_predict_batch_match_oracle(model_dir, strategy):
    cfg, mm, ep = _stack(model_dir, strategy)
    assert mm.engine_slot("xgboost_primary") >= 0 and mm.engine_slot("isolation_forest") >= 0
    # the LSTM file is absent: DummyModel whose tensorflow predict raises -> dropped, as in the reference
    assert mm.is_model_loaded("lstm_sequential") and mm.engine_slot("lstm_sequential") < 0
    xgb, ifm = _oracle_models(model_dir)
    cases = [c for c in json.loads((GOLDEN / "feature_processor_cases.json").read_text()) if "vector" in c][:200]
    processed = [FR.process_features(c["raw"]) for c in cases]
    X = np.array([c["vector"] for c in cases])
    px, _, _ = oracle.xgb_predict(xgb, X)
    pi, _, _ = oracle.iforest_predict(ifm, X)
    w = ep.model_weights
    batch = asyncio.run(ep.predict_batch(processed))
    for i, (p, r) in enumerate(zip(processed, batch)):
        fp, conf, dec, risk = S.blend_row(["xgboost_primary", "isolation_forest"], [float(px[i]), float(pi[i])], w,
                                          strategy)
        assert abs(r["fraud_probability"] - fp) <= 1e-5
        assert r["decision"] == dec or abs(fp - 0.6) < 1e-6 or abs(fp - 0.8) < 1e-6 or abs(fp - 0.95) < 1e-6
        assert r["risk_level"] == risk or min(abs(fp - t) for t in (0.3, 0.6, 0.8, 0.95)) < 1e-6
        assert set(r["model_predictions"]) == {"xgboost_primary", "isolation_forest"}
        single = asyncio.run(ep.predict(dict(p, transaction_id=f"{strategy}-{i}")))
        assert single["fraud_probability"] == r["fraud_probability"]
        assert single["decision"] == r["decision"] and single["risk_level"] == r["risk_level"]
        assert single["model_predictions"] == r["model_predictions"]


def test_model_manager_contract(model_dir):
    cfg, mm, ep = _stack(model_dir)
    X = np.zeros((3, 64))
    with pytest.raises(ValueError):
        asyncio.run(mm.predict("graph_neural", X))  # disabled -> never loaded
    p = asyncio.run(mm.predict("xgboost_primary", X))
    assert p.dtype == np.float32 and p.shape == (3,)
    with pytest.raises(ValueError):  # XGBoost: more columns than the booster's num_feature
        asyncio.run(mm.predict("xgboost_primary", np.zeros((2, 70))))
    with pytest.raises(TypeError):  # the reference's DummyModel tensorflow path
        asyncio.run(mm.predict("lstm_sequential", X))
    asyncio.run(mm.reload_model("xgboost_primary"))
    assert mm.is_model_loaded("xgboost_primary") and mm.engine_slot("xgboost_primary") >= 0
    info = mm.get_model_info()
    assert info["total_models"] == 3
    asyncio.run(mm.cleanup())
    assert not mm.is_model_loaded("xgboost_primary")


def test_wide_vectors_drop_models_per_row(model_dir):
    """A Flink `features` sub-dict can push a row's vector past 64 columns. The reference scores each
    transaction's own vector: XGBoost rejects > num_feature columns and sklearn's IsolationForest any
    width != n_features_in_, so for THAT row both are dropped (-> "No model predictions available"), while
    the batch's 64-wide rows keep both models (per-row, not per-batch, width handling)."""
    cfg, mm, ep = _stack(model_dir)
    xgb, ifm = _oracle_models(model_dir)
    cases = [c for c in json.loads((GOLDEN / "feature_processor_cases.json").read_text()) if "vector" in c][:20]
    processed = [FR.process_features(c["raw"]) for c in cases]
    X = np.array([c["vector"] for c in cases])
    narrow = asyncio.run(ep.predict_batch(processed))
    wide = dict(processed[0], features={f"flink_{k}": 0.25 for k in range(40)})
    from fdengine.ensemble import prepare_features
    assert prepare_features(wide).shape[1] > 64
    with pytest.raises(ValueError):
        asyncio.run(ep.predict(dict(wide, transaction_id="wide-single")))  # every model dropped
    with pytest.raises(ValueError):
        asyncio.run(ep.predict_batch(processed[:5] + [wide]))  # that row has no model, as predict() raises
    # a 64-wide row whose sub-dict keeps it <= 64 columns is unaffected; the others score as before
    px, _, _ = oracle.xgb_predict(xgb, X)
    pi, _, _ = oracle.iforest_predict(ifm, X)
    for i, r in enumerate(narrow):
        fp, _, _, _ = S.blend_row(["xgboost_primary", "isolation_forest"], [float(px[i]), float(pi[i])],
                                  ep.model_weights)
        assert abs(r["fraud_probability"] - fp) <= 1e-5
    with pytest.raises(ValueError):  # IsolationForest: any width != n_features_in_
        asyncio.run(mm.predict("isolation_forest", np.zeros((2, 63))))


def test_predict_runs_off_the_event_loop(model_dir):
    """ModelManager.predict awaits the GPU call in an executor: other coroutines progress meanwhile."""
    cfg, mm, ep = _stack(model_dir)
    X = np.zeros((4096, 64))
    ticks = []

    async def ticker():
        for _ in range(50):
            ticks.append(1)
            await asyncio.sleep(0)

    async def main():
        t = asyncio.create_task(ticker())
        p = await mm.predict("xgboost_primary", X)
        await t
        return p

    p = asyncio.run(main())
    assert p.shape == (4096,) and len(ticks) == 50
