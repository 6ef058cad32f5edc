"""Pipelined stream (config 3/4) from a rocprofv3 kernel-trace CSV: for each fused ensemble launch, the idle time
since the previous ensemble launch ended and since the feature bucket pass it depends on ended, plus the kernels
that ran in between (the critical path of the step is ensemble -> wait -> ensemble)."""
import csv
import statistics
import sys
from collections import Counter


def main(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    ens = [r for r in rows if "ensemble_kernel" in r[2]]
    lean = [r for r in rows if "feat_bucket_lean" in r[2]]
    gaps_prev, gaps_dep, between = [], [], Counter()
    for a, b in zip(ens, ens[1:]):
        g = (b[0] - a[1]) / 1e3
        if g > 30:  # not back-to-back steps
            continue
        gaps_prev.append(g)
        dep = [l for l in lean if l[1] <= b[0] and l[0] >= a[0] - 200_000]
        if dep:
            gaps_dep.append((b[0] - dep[-1][1]) / 1e3)
        for r in rows:
            if a[1] <= r[0] < b[0]:
                between[r[2][:60]] += 1
    dur = [(e - s) / 1e3 for s, e, _ in ens]
    print(f"ensemble launches {len(ens)}, median duration {statistics.median(dur):.2f} us")
    print(f"back-to-back pairs {len(gaps_prev)}: idle between ensembles median {statistics.median(gaps_prev):.2f} "
          f"p90 {sorted(gaps_prev)[int(0.9 * len(gaps_prev))]:.2f} us")
    if gaps_dep:
        print(f"  ensemble start - its lean bucket end: median {statistics.median(gaps_dep):.2f} us "
              f"(negative: the bucket pass ended earlier than that... n/a)")
    ld = [(e - s) / 1e3 for s, e, _ in lean]
    if ld:
        print(f"lean bucket launches {len(ld)}, median duration {statistics.median(ld):.2f} us")
    print("kernels starting in the idle gaps:", dict(between.most_common(8)))


if __name__ == "__main__":
    main(sys.argv[1])


def timeline(path, k0=100, count=4):
    """kernels of `count` consecutive steps from the k0-th ensemble launch, in us from its start"""
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    ens = [r for r in rows if "ensemble_kernel" in r[2]]
    t0, t1 = ens[k0][0], ens[k0 + count][0]
    for s, e, k in rows:
        if t0 - 100_000 <= s < t1:
            print(f"  {(s - t0) / 1e3:9.2f} {(e - t0) / 1e3:9.2f}  {k[:70]}")


if __name__ == "__main__" and len(sys.argv) > 2:
    timeline(sys.argv[1])
