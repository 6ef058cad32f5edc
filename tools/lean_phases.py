#!/usr/bin/env python3
"""Phase cycles (s_memtime) of the pipelined lean bucket kernel, from the stamps bench.py saves with the profiling
library (FD_BENCH_DUMP_FPROF=prefix, FDENGINE_LIB=lib/libfdengine_prof.so): per workgroup start, keys loaded,
sorted, cards done (thread 0) and each wave's end of its card loop.

usage: python tools/lean_phases.py prefix.*.npy [workgroups=512]"""
import sys

import numpy as np


def main(paths, nb=512):
    for path in paths:
        p = np.load(path).reshape(4096, 8)[:nb].astype(np.float64)
        ok = (p[:, 1] > 0) & (p[:, 2] > p[:, 1])
        p = p[ok]
        t0 = p[:, 0].min()
        print(f"{path}: {len(p)} fast-path workgroups; start spread (cycles) median {np.median(p[:, 0] - t0):.0f} "
              f"max {(p[:, 0] - t0).max():.0f}; whole launch {(p[:, 4:8].max() - t0):.0f}")
        for k, nm in enumerate(["keys load", "sort", "cards (thread 0)"]):
            d = p[:, k + 1] - p[:, k]
            print(f"  {nm:16s} median {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}  max {d.max():8.0f}")
        w = p[:, 4:8] - p[:, 2:3]
        print(f"  per-wave card loop median {np.median(w):8.0f}  p90 {np.percentile(w, 90):8.0f}  max {w.max():8.0f}")
        tot = p[:, 4:8].max(axis=1) - p[:, 0]
        print(f"  workgroup total  median {np.median(tot):8.0f}  p90 {np.percentile(tot, 90):8.0f}")
        cpath = path.replace(".npy", ".c.npy")
        try:
            c = np.load(cpath).reshape(4096, 4)[:nb].astype(np.float64)[ok]
        except OSError:
            continue
        good = (c[:, 0] > p[:, 2]) & (c[:, 2] >= c[:, 1]) & (c[:, 1] >= c[:, 0])
        c, q = c[good], p[good]
        for nm, d in (("card: header+prep in", c[:, 0] - q[:, 2]), ("card: velocity/ring", c[:, 1] - c[:, 0]),
                      ("card: emit (vector)", c[:, 2] - c[:, 1]), ("card: rest to end", q[:, 3] - c[:, 2])):
            print(f"  {nm:22s} median {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a.endswith(".npy") and not a.endswith(".c.npy")]
    main(args)
