#!/usr/bin/env python3
"""Per-wave cycle split of the fused ensemble kernel (profiling build lib/libfdengine_prof.so,
-DFD_FOREST_PROFILE, s_memtime stamps): prologue (binning), chunk-loop top (leaf stores, DMA issue, owner
add), walk (+ leaf-value loads), DMA wait + barrier. Workload: the bench's models (XGBoost 500 x depth 8 +
IsolationForest 100) over B random 64-wide vectors."""
import ctypes as C
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
os.environ.setdefault("FDENGINE_LIB", str(REPO / "realtime-fraud-detection_amd" / "lib" / "libfdengine_prof.so"))
sys.path[:0] = [str(REPO), str(REPO / "realtime-fraud-detection_amd")]
import numpy as np

import fdengine
from fdengine import FraudEngine, _native, iforest_from_sklearn, synth, xgboost_from_json_doc

B = int(os.environ.get("B", 65536))
T = int(os.environ.get("TREES", 500))
if os.environ.get("DATA", "bench") == "bench":  # the bench's models and engine-made scoring vectors
    import bench
    xgb, ifm = bench.fit_models(0, T, 8, 1, 16)
    spop = synth.population(20000, 500, seed=21)
    stx = synth.txn_stream(spop, B, seed=22, rate_per_s=20.0)
    scratch = fdengine.FraudEngine(0)
    scratch.state_init(1 << 16, 1, 16)
    scratch.load_users(spop["users"]["key"], spop["users"]["avg_amount"], spop["users"]["account_age_days"],
                       spop["users"]["device_fp"])
    scratch.load_merchants(spop["merchants"]["fraud_rate"], spop["merchants"]["risk_multiplier"])
    X = scratch.features(stx)
    scratch.close()
else:
    Xr = synth.feature_matrix(8192, 64, seed=1)
    xgb = xgboost_from_json_doc(synth.xgboost_doc(T, 8, 64, Xr, seed=2, p_leaf=0.0))
    ifm = iforest_from_sklearn(synth.isolation_forest(Xr.astype(np.float64), n_estimators=100))
    X = synth.feature_matrix(B, 64, seed=3)
eng = fdengine.FraudEngine(0)
eng.load_forest(0, xgb)
eng.load_forest(1, ifm)
params = FraudEngine.blend_params([0.4 / 0.45, 0.05 / 0.45], [1.0, 0.5])
for _ in range(3):
    eng.score_matrix(params, [0, 1], X)
buf = np.zeros(4 * 256 * 16 * 16, np.uint64)  # the profile buffers of the last 4 launches
_native.lib.fd_debug_ens_profile.argtypes = [C.c_void_p, C.c_int]
assert _native.lib.fd_debug_ens_profile(buf.ctypes.data, buf.size) == 0
newest = (_native.lib.fd_debug_ens_profile_next() + 3) % 4
nb = min(256, (B + 255) // 256)
p = buf.reshape(4, 256, 16, 16)[newest, :nb].astype(np.float64)
tot = p[:, :, 5] - p[:, :, 4]
print(f"{nb} workgroups x 16 waves; cycles per wave (median / p10 / p90):")
for k, nm in enumerate(["prologue", "loop top", "walk+leaf", "wait+barrier"]):
    v = p[:, :, k]
    print(f"  {nm:13s} {np.median(v):9.0f} {np.percentile(v, 10):9.0f} {np.percentile(v, 90):9.0f}"
          f"   share {np.median(v / tot):.3f}")
print(f"  {'total':13s} {np.median(tot):9.0f} {np.percentile(tot, 10):9.0f} {np.percentile(tot, 90):9.0f}")
dm = p[:, :, 13][:, :4]  # tree group 0 (the chunk owner) waits for its LDS-DMA before the barrier
print(f"  owner DMA wait (group 0, inside wait+barrier): median {np.median(dm):.0f} p90 {np.percentile(dm, 90):.0f}")
wk = p[:, :, 2]
print("  walk+leaf by tree group (median):", [float(np.median(wk[:, g * 4:(g + 1) * 4])) for g in range(4)])
st = p[:, :, 6:13]
print("  prologue marks (cycles from wave start, median): raw+barrier, then per pass (tables staged, binned):",
      [float(np.median(st[:, :, k])) for k in range(7)])
