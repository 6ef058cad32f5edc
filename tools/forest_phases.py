#!/usr/bin/env python3
"""Phase-cycle breakdown of forest_kernel3 on the config-2 workload (profiling build of the engine,
lib/libfdengine_prof.so, -DFD_FOREST_PROFILE). Per wave of the first 256 workgroups: prologue, walk,
leaf store, owner sum, barrier wait, total (s_memtime cycles)."""
import ctypes as C
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
os.environ.setdefault("FDENGINE_LIB", str(REPO / "realtime-fraud-detection_amd" / "lib" / "libfdengine_prof.so"))
sys.path[:0] = [str(REPO), str(REPO / "realtime-fraud-detection_amd")]
import numpy as np
import torch

import fdengine
from fdengine import _native, synth

B = int(os.environ.get("B", 65536)); F = int(os.environ.get("F", 50)); T = int(os.environ.get("T", 500)); D = 8
X = synth.feature_matrix(B, F, seed=1000)
forest = fdengine.xgboost_from_json_doc(synth.xgboost_doc(T, D, F, synth.feature_matrix(2048, F, seed=7), seed=8))
eng = fdengine.FraudEngine(0)
eng.load_forest(0, forest)
dX = torch.from_numpy(X).cuda()
dp = torch.empty(B, dtype=torch.float64, device="cuda")
eng.set_stream(torch.cuda.current_stream().cuda_stream)
eng.set_option("forest_kernel", int(os.environ.get("VARIANT", 2)))
for _ in range(5):
    eng.predict_device(0, dX.data_ptr(), B, F, dp.data_ptr())
torch.cuda.synchronize()
lib = _native.lib
buf = np.zeros(256 * 16 * 8, np.uint64)
lib.fd_debug_forest_profile.argtypes = [C.c_void_p, C.c_int]
assert lib.fd_debug_forest_profile(buf.ctypes.data, buf.size) == 0
p = buf.reshape(256, 16, 8).astype(np.float64)
names = ["prologue", "walk", "leaf", "owner", "barrier", "total"]
print("median cycles per wave (s_memtime):")
for i, nm in enumerate(names):
    print(f"  {nm:9s} {np.median(p[:, :, i]):10.0f}   p10 {np.percentile(p[:, :, i], 10):10.0f}  p90 {np.percentile(p[:, :, i], 90):10.0f}")
start = p[:, 0, 6]
print("workgroup start spread (cycles):", float(start.max() - start.min()))
# per wave index (0..15; wave w: tree group w >> 2, transaction group w & 3; SIMD = w mod 4 under the
# usual round-robin placement): is the walk's spread systematic?
print("walk / barrier median per wave index:")
for w in range(16):
    print(f"  wave {w:2d}  walk {np.median(p[:, w, 1]):9.0f}  barrier {np.median(p[:, w, 4]):9.0f}  owner {np.median(p[:, w, 3]):8.0f}")
