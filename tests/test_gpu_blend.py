"""GPU parity of the ensemble epilogue (fd_blend_*) against the pure-Python restatement of
EnsemblePredictor (oracle/scoring_ref.py, itself pinned to the imported reference by golden vectors).
f64 arithmetic in the reference's order -> outputs must be identical, not merely close."""
import numpy as np
import pytest

from fdengine import FraudEngine
from fdengine._native import DECISIONS, RISK_LEVELS
from oracle import scoring_ref as S

pytestmark = pytest.mark.gpu

NAMES = ["xgboost_primary", "lstm_sequential", "isolation_forest"]
RAW_W = {"xgboost_primary": 0.4, "lstm_sequential": 0.25, "isolation_forest": 0.05}


def _probs(n, seed):
    rng = np.random.default_rng(seed)
    cols = []
    for m in range(3):
        p = rng.random(n)
        p[rng.random(n) < 0.05] = rng.choice([0.0, 1.0, 0.5, -0.3, 1.7, np.nan, 0.95, 0.8, 0.6, 0.3], 1)[0]
        cols.append(p)
    return cols


@pytest.mark.parametrize("strategy,code", [("weighted_average", 0), ("voting", 1), ("stacking", 2)])
@pytest.mark.parametrize("present", [(1, 1, 1), (1, 0, 1), (0, 0, 1)])
def test_blend_matches_reference_restatement(engine, strategy, code, present):
    n = 5000
    w = S.normalized_weights(RAW_W)
    cols = _probs(n, seed=100 * code + 10 * present[0] + 2 * present[1] + present[2])
    params = FraudEngine.blend_params([w[k] for k in NAMES], [S.CONF_MULT[k] for k in NAMES], strategy=code)
    probs = [c if ok else None for c, ok in zip(cols, present)]
    fp, conf, dec, risk = engine.blend(params, probs)
    for i in range(n):
        rfp, rconf, rdec, rrisk = S.blend_row(NAMES, [None if p is None else p[i] for p in probs], w, strategy)
        assert fp[i] == rfp or (np.isnan(fp[i]) and np.isnan(rfp)), (i, fp[i], rfp)
        assert conf[i] == rconf, (i, conf[i], rconf)
        assert DECISIONS[dec[i]] == rdec
        assert RISK_LEVELS[risk[i]] == rrisk
