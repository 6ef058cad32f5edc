#!/usr/bin/env python3
"""A/B of engine options on the fused ensemble kernel: the bench's models (XGBoost 500 x 8 + IsolationForest
100, tools/ens_phases.py) over B engine-made scoring vectors; kernel time from the engine's HIP events
(FD_TIMING_ENSEMBLE), arms interleaved round-robin so clock drift hits every arm alike.

    OPTS="ensemble_owner=0;ensemble_owner=1" python tools/ens_ab.py
"""
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "realtime-fraud-detection_amd")]
import numpy as np

import bench
import fdengine
from fdengine import FraudEngine, synth
from fdengine._native import FD_TIMING_ENSEMBLE

B = int(os.environ.get("B", 65536))
ROUNDS = int(os.environ.get("ROUNDS", 12))
REPS = int(os.environ.get("REPS", 10))
arms = [a for a in os.environ.get("OPTS", "ensemble_owner=0;ensemble_owner=1").split(";") if a]

xgb, ifm = bench.fit_models(0, 500, 8, 1, 16)
spop = synth.population(20000, 500, seed=21)
stx = synth.txn_stream(spop, B, seed=22, rate_per_s=20.0)
scratch = fdengine.FraudEngine(0)
scratch.state_init(1 << 16, 1, 16)
U, M = spop["users"], spop["merchants"]
scratch.load_users(U["key"], U["avg_amount"], U["account_age_days"], U["device_fp"])
scratch.load_merchants(M["fraud_rate"], M["risk_multiplier"])
X = scratch.features(stx)
scratch.close()
eng = fdengine.FraudEngine(0)
eng.load_forest(0, xgb)
eng.load_forest(1, ifm)
params = FraudEngine.blend_params([0.4 / 0.45, 0.05 / 0.45], [1.0, 0.5])


def apply(arm):
    for kv in arm.split(","):
        k, v = kv.split("=")
        eng.set_option(k.strip(), int(v))


ref = None
times = {a: [] for a in arms}
for r in range(ROUNDS):
    for a in arms:
        apply(a)
        eng.read_timing()
        eng.set_timing(True)
        for _ in range(REPS):
            out = eng.score_matrix(params, [0, 1], X)
        eng.set_timing(False)
        ms, n = eng.read_timing(FD_TIMING_ENSEMBLE)
        assert n == REPS, (a, n)
        times[a].append(ms / n * 1e3)
        if ref is None:
            ref = out
        else:
            for u, v in zip(out, ref):
                np.testing.assert_array_equal(u, v)
for a in arms:
    t = np.array(times[a][2:])
    print(f"{a:40s} median {np.median(t):8.2f} us   min {t.min():8.2f}   max {t.max():8.2f}")
print("outputs identical across arms")
