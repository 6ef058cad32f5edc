"""Per-kernel duration and launch gap from a rocprofv3 kernel-trace CSV.

For every kernel name: launches, median duration, and the median gap between the previous kernel's end and its
start (same queue order, whole trace sorted by start). The longest run of back-to-back launches with the same
repeating kernel sequence dominates the medians when the bench's timed region is the bulk of the trace.
"""
import csv
import statistics
import sys
from collections import defaultdict


def main(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    dur, gap = defaultdict(list), defaultdict(list)
    for i, (s, e, k) in enumerate(rows):
        dur[k].append((e - s) / 1e3)
        if i:
            g = (s - rows[i - 1][1]) / 1e3
            if g < 50:  # skip host-side pauses (latency loop, setup)
                gap[k].append(g)
    print(f"{'kernel':70s} {'n':>6s} {'dur_med_us':>10s} {'gap_med_us':>10s}")
    for k in sorted(dur, key=lambda k: -len(dur[k]) * statistics.median(dur[k])):
        if len(dur[k]) < 50:
            continue
        gm = statistics.median(gap[k]) if gap[k] else float("nan")
        print(f"{k[:70]:70s} {len(dur[k]):6d} {statistics.median(dur[k]):10.2f} {gm:10.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
