#!/usr/bin/env python3
"""Phase-cycle breakdown of the feature bucket kernel (profiling build lib/libfdengine_prof.so,
-DFD_FOREST_PROFILE): per workgroup s_memtime at start, keys loaded, sorted, short segments done, plus each
wave's end of its short-segment loop. Workload: config4-like (CARDS cards, routed SoA batch of B)."""
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
from fdengine._native import TXN_FIELDS

B = int(os.environ.get("B", 65536))
CARDS = int(os.environ.get("CARDS", 10_000_000))
K = int(os.environ.get("K", 16))
merch = synth.merchants_table(5000, seed=100)
own = synth.owned_cards(CARDS, 0, 1, seed=42)
cap = 1
while cap < int(CARDS * 1.6) + 65536:
    cap *= 2
eng = fdengine.FraudEngine(0)
eng.set_stream(torch.cuda.current_stream().cuda_stream)
eng.state_init(cap, 1, K)
eng.load_users(own["key"], own["avg_amount"], own["account_age_days"], own["device_fp"])
eng.load_merchants(merch["fraud_rate"], merch["risk_multiplier"])
tx = synth.txn_stream_cards(CARDS, merch, 8 * B, seed=200, card_seed=42, rate_per_s=2000.0)
dev = {f: torch.from_numpy(np.ascontiguousarray(tx[f])).cuda() for f in TXN_FIELDS}
vec = torch.empty((B, 64), dtype=torch.float32, device="cuda")
el = {f: tx[f].dtype.itemsize for f in TXN_FIELDS}
for b in range(8):
    eng.features_device({f: t.data_ptr() + b * B * el[f] for f, t in dev.items()}, B, vec.data_ptr())
torch.cuda.synchronize()
nb = 1
while nb * 128 < B:
    nb *= 2
buf = np.zeros(4096 * 8, np.uint64)
_native.lib.fd_debug_feat_profile.argtypes = [C.c_void_p, C.c_int]
assert _native.lib.fd_debug_feat_profile(buf.ctypes.data, buf.size) == 0
p = buf.reshape(4096, 8)[:nb].astype(np.float64)
t0 = p[:, 0].min()
print(f"{nb} workgroups; cycles relative to the first workgroup start (median / p90 / max):")
for k, nm in enumerate(["start", "keys loaded", "sorted", "short done"]):
    v = p[:, k] - t0
    print(f"  {nm:12s} {np.median(v):9.0f} {np.percentile(v, 90):9.0f} {v.max():9.0f}")
for k, nm in enumerate(["keys load", "sort", "short segs"]):
    d = p[:, k + 1] - p[:, k]
    print(f"  phase {nm:11s} {np.median(d):9.0f} {np.percentile(d, 90):9.0f} {d.max():9.0f}")
w = p[:, 4:8] - p[:, 2:3]
print("  per-wave short-loop time after sort: median", np.median(w), "p90", np.percentile(w, 90))
