"""One engine driven from several host threads (include/fdengine.h: every entry point holds the engine's lock).

The reference serialises on one asyncio loop (ml/main.py:337-344); the drop-in runs ModelManager.predict in a
worker thread (model_manager.py:279-307 semantics) while predict_batch, loads and reloads stay on the loop's thread.
Here two threads share one engine: one scores through the host API (engine staging buffers), the other scores
another batch and reloads its forest over and over. Every result must equal the single-threaded one."""
import threading

import numpy as np
import pytest

from fdengine import FraudEngine, iforest_from_sklearn, synth, xgboost_from_json_doc

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
def test_concurrent_predict_and_reload():
    X = synth.feature_matrix(6000, 64, seed=31)
    xgb = xgboost_from_json_doc(synth.xgboost_doc(100, 8, 64, X, seed=32))
    ifm = iforest_from_sklearn(synth.isolation_forest(X.astype(np.float64), n_estimators=30))
    eng = FraudEngine(0)
    try:
        eng.load_forest(0, xgb)
        eng.load_forest(1, ifm)
        want_x = eng.predict(0, X[:3000])
        want_i = eng.predict(1, X[3000:])
        errors = []

        def scorer():
            try:
                for _ in range(60):
                    assert np.array_equal(eng.predict(0, X[:3000]), want_x)
            except Exception as e:  # reported below
                errors.append(e)

        def reloader():
            try:
                for _ in range(30):
                    eng.load_forest(1, ifm)
                    assert np.array_equal(eng.predict(1, X[3000:]), want_i)
            except Exception as e:
                errors.append(e)

        ts = [threading.Thread(target=scorer), threading.Thread(target=reloader)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=240)
        assert not any(t.is_alive() for t in ts), "a thread did not finish"
        assert not errors, errors[0]
    finally:
        eng.close()
