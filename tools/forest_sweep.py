#!/usr/bin/env python3
"""A/B the forest kernel variants on the config-2 workload in ONE process, interleaved rounds
(cdna_hip_programming.md rule 24). Prints per-variant median/min kernel time (HIP events)."""
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "realtime-fraud-detection_amd")]
import numpy as np
import torch

import fdengine
from fdengine import synth

B = int(os.environ.get("B", 65536)); F = 50; T = int(os.environ.get("T", 500)); D = 8
variants = [int(v) for v in os.environ.get("VARIANTS", "1,2").split(",")]
rounds, reps = 5, 20
X = synth.feature_matrix(4 * B, F, seed=1000)
if os.environ.get("IF"):  # the config-3 IsolationForest (100 trees, max_samples 256, f64 leaves)
    forest = fdengine.iforest_from_sklearn(
        synth.isolation_forest(synth.feature_matrix(20000, F, seed=7).astype(np.float64), n_estimators=100))
else:
    forest = fdengine.xgboost_from_json_doc(synth.xgboost_doc(T, D, F, synth.feature_matrix(2048, F, seed=7), seed=8))
eng = fdengine.FraudEngine(0)
eng.load_forest(0, forest)
print("forest", eng.forest_info(0))
dX = torch.from_numpy(X).cuda()
dp = torch.empty(4 * B, dtype=torch.float64, device="cuda")
eng.set_stream(torch.cuda.current_stream().cuda_stream)
res = {v: [] for v in variants}
ref = None
for r in range(rounds):
    for v in variants:
        eng.set_option("forest_kernel", v)
        for i in range(3):
            eng.predict_device(0, dX.data_ptr() + (i % 4) * B * F * 4, B, F, dp.data_ptr() + (i % 4) * B * 8)
        torch.cuda.synchronize()
        eng.read_timing(); eng.set_timing(True)
        for i in range(reps):
            eng.predict_device(0, dX.data_ptr() + (i % 4) * B * F * 4, B, F, dp.data_ptr() + (i % 4) * B * 8)
        torch.cuda.synchronize()
        eng.set_timing(False)
        ms, n = eng.read_timing(1 if os.environ.get("IF") else 0)
        res[v].append(ms / n * 1e3)
        out = dp[:B].cpu().numpy()
        if ref is None:
            ref = out
        assert np.array_equal(out, ref), f"variant {v} output differs"
for v in variants:
    a = np.array(res[v])
    print(f"variant {v}: median {np.median(a):.1f} us  min {a.min():.1f} us  -> {B / np.median(a) * 1e6 / 1e6:.1f} M txn/s")
