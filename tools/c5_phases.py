#!/usr/bin/env python3
"""Workgroup timeline of one config-5 step (1 k latency batch) from the profiling build (lib/libfdengine_prof.so,
-DFD_FOREST_PROFILE, FD_TL stamps in the 100 MHz GPU clock): per kernel the first workgroup start, the last
workgroup end, the median workgroup time and its marks, and the gap from the previous kernel's last end.

Runs bench.py's Config5 workload for a few steps (default engine options; extra --engine-option args pass through),
then one step alone after a synchronize, and reads the stamps that step left."""
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

NAMES = {0: "feat_slot", 1: "feat_bucket", 2: "lstm_kernel4", 3: "split_bin_pair", 4: "split_walk_pair",
         5: "split_sum_pair_blend"}
MARKS = {2: ("staged", "recurrence done"), 5: ("leaves loaded", "summed")}


def main():
    extra = sys.argv[1:]
    args = bench.parse_args(["--workload", "config5", "--steps", "40", "--warmup", "2", "--latency-iters", "0",
                             "--alone-iters", "0", "--loaded-iters", "0", "--timing-steps", "0",
                             "--parity-batches", "0"] + extra)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = fdengine.FraudEngine(0)
    for kv in args.engine_option:
        k, v = kv.split("=")
        eng.set_option(k.strip(), int(v))
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    wl = bench.WORKLOADS["config5"](args, 0, dev, eng)
    wl.parity_done = True
    def stamps():
        buf = np.zeros(8 * 1024 * 4, np.uint64)
        tot = np.zeros_like(buf)
        for fn in ("fd_debug_tl_feat", "fd_debug_tl_lstm", "fd_debug_tl_forest"):
            f = getattr(_native.lib, fn)
            f.argtypes = [C.c_void_p]
            buf[:] = 0
            assert f(buf.ctypes.data) == 0
            tot = np.maximum(tot, buf)
        return tot.reshape(8, 1024, 4)

    reps = []
    for rep in range(5):
        for i in range(4):
            wl.step(i)
        torch.cuda.synchronize()
        before = stamps()
        wl.step(0)  # the step whose stamps are read: nothing else queued around it
        torch.cuda.synchronize()
        after = stamps()
        # only the workgroups this step ran (a stamp left by an earlier, larger launch is unchanged)
        fresh = after[:, :, 0] != before[:, :, 0]
        q = after.astype(np.float64)
        q[~fresh] = 0.0
        reps.append(q)
    # the last repetition's stamps, ns relative to the step's first stamp
    p = reps[-1]
    order = []
    for kid in NAMES:
        live = p[kid, :, 0] > 0
        if live.any():
            order.append((p[kid, live, 0].min(), kid))
    order.sort()
    t0 = order[0][0]
    print(f"{'kernel':22s} {'wgs':>5s} {'first start':>11s} {'last end':>9s} {'span':>7s} {'gap':>6s} "
          f"{'wg med':>7s}  marks (median from start)")
    prev_end = None
    for _, kid in order:
        live = p[kid, :, 0] > 0
        s, e = p[kid, live, 0], p[kid, live, 3]
        span = (e.max() - s.min()) * 10 / 1e3
        gap = "" if prev_end is None else f"{(s.min() - prev_end) * 10 / 1e3:6.2f}"
        marks = ""
        for k, nm in enumerate(MARKS.get(kid, ()), start=1):
            m = p[kid, live, k]
            ok = m > 0
            if ok.any():
                marks += f"  {nm} {np.median(m[ok] - s[ok]) * 10 / 1e3:.2f}"
        print(f"{NAMES[kid]:22s} {live.sum():5d} {(s.min() - t0) * 10 / 1e3:11.2f} {(e.max() - t0) * 10 / 1e3:9.2f} "
              f"{span:7.2f} {gap:>6s} {np.median(e - s) * 10 / 1e3:7.2f} {marks}")
        prev_end = e.max()
    # the bucket kernel's own phase stamps (s_memtime cycles, FD_FSTAMP): start, keys loaded, sorted, short done
    fb = np.zeros(4096 * 8, np.uint64)
    _native.lib.fd_debug_feat_profile.argtypes = [C.c_void_p, C.c_int]
    assert _native.lib.fd_debug_feat_profile(fb.ctypes.data, fb.size) == 0
    nb = int((p[1, :, 0] > 0).sum())
    fq = fb.reshape(4096, 8)[:nb].astype(np.float64)
    for k, nm in enumerate(["keys load", "sort", "short segs"]):
        d = fq[:, k + 1] - fq[:, k]
        print(f"  bucket phase {nm:11s} cycles median {np.median(d):8.0f}  max {d.max():8.0f}")
    steps = []
    for q in reps:
        st = [q[k, q[k, :, 0] > 0, 0].min() for k in NAMES if (q[k, :, 0] > 0).any()]
        en = [q[k, q[k, :, 3] > 0, 3].max() for k in NAMES if (q[k, :, 3] > 0).any()]
        steps.append((max(en) - min(st)) * 10 / 1e3)
    print("step span (first start -> last end, us) over", len(steps), "repetitions:", [round(x, 2) for x in steps])


if __name__ == "__main__":
    main()
