#!/usr/bin/env python3
"""Where the config-4 step's time goes outside the kernels: the bench's own workload object (10 M cards by
default), K steps timed wall-clock with the engine's per-kernel HIP-event timing on and off, interleaved.

    CARDS=10000000 STEPS=200 python tools/step_gap.py
"""
import argparse
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "realtime-fraud-detection_amd")]
import torch

import bench
import fdengine

steps = int(os.environ.get("STEPS", 200))
args = argparse.Namespace(gpus=1, steps=steps, warmup=20, workload="config4", batch=65536, trees=500, depth=8,
                          features=50, pool=8, cards=int(os.environ.get("CARDS", 10_000_000)), window="sliding",
                          ring_k=16, cpu_seconds=0.0, no_cpu_baseline=True, latency_iters=0, parity_batches=0)
args.warmup, args.latency_iters = 20, 0
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
eng = fdengine.FraudEngine(0)
stream = torch.cuda.current_stream(dev)
eng.set_stream(stream.cuda_stream)
args.steps = 8 * steps + 40  # enough resident batches for every arm
wl = bench.WORKLOADS["config4"](args, 0, dev, eng)
for i in range(20):
    wl.step(i)
torch.cuda.synchronize()
res = {"timing on": [], "timing off": []}
for rep in range(3):
    for arm in res:
        eng.set_timing(arm == "timing on")
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(steps):
            wl.step(i)
        torch.cuda.synchronize()
        res[arm].append((time.perf_counter() - t) / steps * 1e6)
        eng.set_timing(False)
        tm = eng.read_timing()
        if arm == "timing on":
            print("kernel averages (us):", {k: round(v[0] / max(v[1], 1) * 1e3, 2) for k, v in tm.items() if v[1]},
                  flush=True)
for arm, v in res.items():
    print(f"{arm:12s}: step {min(v):7.2f} us (min of {len(v)}), all {[round(x, 2) for x in v]}", flush=True)
eng.close()
