#!/usr/bin/env python3
"""Per-wave cycle split of the fused ensemble kernel inside the pipelined stream (profiling build
lib/libfdengine_prof.so, -DFD_FOREST_PROFILE): the bench's config-4 workload (warm stream; CARDS cards, default
10M to keep setup short) stepped through ShardedScorer -> fd_score_batch_pipelined, then the profile of the
last launches that ran BESIDE the next batch's feature kernels, against launches run one at a time (alone).
Phases: prologue (row loads, table staging, binning), chunk-loop top, walk (+ leaf stores), DMA wait + barrier.

  python tools/ens_phases_pipe.py          (build first: python realtime-fraud-detection_amd/fdengine/build.py --profile)
"""
import ctypes as C
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
os.environ.setdefault("FDENGINE_LIB", str(REPO / "realtime-fraud-detection_amd" / "lib" / "libfdengine_prof.so"))
sys.path[:0] = [str(REPO), str(REPO / "realtime-fraud-detection_amd")]
import numpy as np
import torch

import bench
import fdengine
from fdengine import _native

SLOTS, NB, NW, NF = 4, 256, 16, 16


def read_profiles():
    buf = np.zeros(SLOTS * NB * NW * NF, np.uint64)
    _native.lib.fd_debug_ens_profile.argtypes = [C.c_void_p, C.c_int]
    assert _native.lib.fd_debug_ens_profile(buf.ctypes.data, buf.size) == 0
    nxt = _native.lib.fd_debug_ens_profile_next()
    p = buf.reshape(SLOTS, NB, NW, NF).astype(np.float64)
    order = [(nxt + k) % SLOTS for k in range(SLOTS)]  # oldest .. newest launch
    return [p[s] for s in order]


def summary(name, ps):
    tot = np.concatenate([(p[:, :, 5] - p[:, :, 4]).ravel() for p in ps])
    print(f"{name}: {len(ps)} launches x {NB} workgroups x {NW} waves; cycles per wave (median / p10 / p90):")
    for k, nm in enumerate(["prologue", "loop top", "walk+leaf", "wait+barrier"]):
        v = np.concatenate([p[:, :, k].ravel() for p in ps])
        sh = np.concatenate([(p[:, :, k] / (p[:, :, 5] - p[:, :, 4])).ravel() for p in ps])
        print(f"  {nm:13s} {np.median(v):9.0f} {np.percentile(v, 10):9.0f} {np.percentile(v, 90):9.0f}   share "
              f"{np.median(sh):.3f}")
    print(f"  {'total':13s} {np.median(tot):9.0f} {np.percentile(tot, 10):9.0f} {np.percentile(tot, 90):9.0f}")
    dm = np.concatenate([p[:, :4, 13].ravel() for p in ps])
    print(f"  owner DMA wait (group 0): median {np.median(dm):.0f} p90 {np.percentile(dm, 90):.0f}")
    wk = [float(np.median(np.concatenate([p[:, g * 4:(g + 1) * 4, 2].ravel() for p in ps]))) for g in range(4)]
    print("  walk+leaf by tree group (median):", wk)
    st = np.concatenate([p[:, :, 6:13] for p in ps], axis=0)
    print("  prologue marks (median):", [float(np.median(st[:, :, k])) for k in range(7)])
    # workgroup start / end times on the GPU-wide 100 MHz clock (s_memrealtime): how late the workgroups of a
    # launch start (waiting for a CU) relative to its first, and the launch's span, in microseconds
    late, span = [], []
    for p in ps:
        t0 = p[:, :, 14].min(axis=1)  # each workgroup's first wave start
        t1 = p[:, :, 15].max(axis=1)
        late.append(np.percentile(t0 - t0.min(), [50, 90, 100]) / 100.0)
        span.append((t1.max() - t0.min()) / 100.0)
    late = np.array(late)
    print(f"  workgroup start after the launch's first (us, median over launches): p50 {np.median(late[:, 0]):.1f} "
          f"p90 {np.median(late[:, 1]):.1f} max {np.median(late[:, 2]):.1f}; launch span {np.median(span):.1f} us")

def main():
    cards = int(os.environ.get("CARDS", 10_000_000))
    steps = int(os.environ.get("STEPS", 40))
    args = bench.parse_args(["--cards", str(cards), "--steps", str(steps + SLOTS + 2), "--warmup", "2", "--latency-iters", "0",
                             "--alone-iters", "0", "--loaded-iters", "0", "--parity-batches", "0"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = fdengine.FraudEngine(0)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    for kv in os.environ.get("OPTS", "").split(","):  # engine options, e.g. OPTS=ensemble_bin_global=1
        if kv:
            k, v = kv.split("=")
            eng.set_option(k.strip(), int(v))
    wl = bench.WORKLOADS["config4"](args, 0, dev, eng)
    for i in range(args.warmup):
        wl.step(i)
    torch.cuda.synchronize()
    # pipelined: the newest launch had no next batch beside it; the three before it did
    for i in range(steps):
        wl.step(i)
    torch.cuda.synchronize()
    pipe = read_profiles()[:-1]
    # alone: one step at a time
    for i in range(SLOTS):
        wl.step(i)
        torch.cuda.synchronize()
    alone = read_profiles()
    summary("beside the next batch's features", pipe)
    summary("alone", alone)
    eng.close()


if __name__ == "__main__":
    main()
