#!/usr/bin/env python3
"""Shader clock and step interval of the fused ensemble kernel over a timed region, on the device's own clocks
(profiling build lib/libfdengine_prof.so, -DFD_FOREST_PROFILE: per launch, wave 0 of workgroups 0 / 64 / 128 / 192
records s_memtime (shader cycles) and s_memrealtime (100 MHz) at its start and end; ensemble.hip g_eclk).

The bench's config-4 workload (warm stream, the bench's default 100 M cards unless CARDS is set), then IDLE seconds
of host-only time (the bench's parity oracle runs there), WARMUP steps, a synchronize, STEPS pipelined steps. Per
block of 20 launches: the shader clock (memtime cycles / realtime ticks), a wave's duration, and the interval between
consecutive launch starts (the device's step time) — does the 20-step region's excess over long runs follow the
clock?

  IDLE=3 STEPS=200 python tools/clock_ramp.py
"""
import ctypes as C
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
os.environ.setdefault("FDENGINE_LIB", str(REPO / "realtime-fraud-detection_amd" / "lib" / "libfdengine_prof.so"))
sys.path[:0] = [str(REPO), str(REPO / "realtime-fraud-detection_amd")]
import numpy as np
import torch

import bench
import fdengine
from fdengine import _native

SLOTS = 1024


def main():
    steps = int(os.environ.get("STEPS", 200))
    warm = int(os.environ.get("WARMUP", 5))
    idle = float(os.environ.get("IDLE", 3))
    argv = ["--steps", str(steps), "--warmup", str(warm), "--latency-iters", "0", "--alone-iters", "0",
            "--loaded-iters", "0", "--parity-batches", "0", "--no-cpu-baseline"]
    if os.environ.get("CARDS"):
        argv += ["--cards", os.environ["CARDS"]]
    args = bench.parse_args(argv)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = fdengine.FraudEngine(0)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    wl = bench.WORKLOADS["config4"](args, 0, dev, eng)
    torch.cuda.synchronize()
    time.sleep(idle)
    for i in range(warm):
        wl.step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        wl.step(warm + i)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    buf = np.zeros(SLOTS * 16, np.uint64)
    _native.lib.fd_debug_ens_clock.argtypes = [C.c_void_p, C.c_int]
    assert _native.lib.fd_debug_ens_clock(buf.ctypes.data, buf.size) == 0
    nxt = _native.lib.fd_debug_ens_clock_next()
    rec = buf.reshape(SLOTS, 4, 4).astype(np.float64)
    n = warm + steps
    idx = [(nxt - n + k) % SLOTS for k in range(n)]
    r = rec[idx]  # launches in order: [launch][workgroup sample][memtime0, memtime1, realtime0, realtime1]
    mhz = (r[:, :, 1] - r[:, :, 0]) / np.maximum(r[:, :, 3] - r[:, :, 2], 1) * 100.0
    dur = (r[:, :, 3] - r[:, :, 2]) / 100.0  # us
    start = r[:, :, 2].min(axis=1) / 100.0
    print(f"host region: {steps} steps, {(t1 - t0) * 1e3 / steps:.4f} ms/step (idle before warmup {idle} s, "
          f"warmup {warm})")
    print("launches      shader MHz (median)  wave us (median)  start-to-start us/step")
    blocks = [(0, warm)] + [(warm + b, min(n, warm + b + 20)) for b in range(0, steps, 20)]
    for a, b in blocks:
        if b - a < 2:
            continue
        iv = np.diff(start[a:b]).mean()
        tag = "warmup" if a == 0 else f"{a - warm:4d}-{b - warm - 1:4d}"
        print(f"{tag:12s}  {np.median(mhz[a:b]):10.0f}          {np.median(dur[a:b]):8.1f}          {iv:8.2f}")
    eng.close()


if __name__ == "__main__":
    main()
