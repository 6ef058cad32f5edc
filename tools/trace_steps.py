"""Per-step GPU timeline of the pipelined stream from a rocprofv3 kernel-trace CSV (config 3/4 bench runs).

Groups the fused ensemble launches into clusters (consecutive launches less than 2 ms apart: the parity batches, the
warm-up, the timed region, the timing loop), prints each cluster's size and span, and for the clusters of the timed
region's size (and the first steps of the longest one) every step: when its slot / bucket / ensemble kernels ran
relative to the cluster's first kernel, and the ensemble's duration and idle gap before it.

usage: python tools/trace_steps.py run_kernel_trace.csv [steps]"""
import csv
import sys


def short(name):
    if name in ("ens", "lean", "slot", "copy", "bucket"):
        return name
    for k, v in (("ensemble_kernel", "ens"), ("feat_bucket_lean", "lean"), ("feat_slot", "slot"),
                 ("pipe_out_copy", "copy"), ("feat_bucket", "bucket")):
        if k in name:
            return v
    return None


def main(path, steps=20):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            if k:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    ens = [r for r in rows if r[2] == "ens"]
    clusters, cur = [], [ens[0]]
    for a, b in zip(ens, ens[1:]):
        if b[0] - a[1] > 2_000_000:
            clusters.append(cur)
            cur = []
        cur.append(b)
    clusters.append(cur)
    print("clusters of ensemble launches (size, span us, us per launch):")
    for c in clusters:
        span = (c[-1][1] - c[0][0]) / 1e3
        print(f"  {len(c):4d}  {span:10.1f}  {span / len(c):8.2f}")
    longest = max(clusters, key=len)
    for c in clusters:
        if len(c) != steps and c is not longest:
            continue
        c0 = c[0][0]
        lo = c0 - 400_000
        hi = c[min(len(c), steps) - 1][1]
        print(f"\ncluster of {len(c)} (first {steps} steps): t0 = first ensemble start - kernels before it shown")
        prev_end = None
        for s, e, k in rows:
            if s < lo or s > hi:
                continue
            gap = f" gap {(s - prev_end) / 1e3:7.2f}" if k == "ens" and prev_end is not None else ""
            print(f"  {k:6s} {(s - c0) / 1e3:9.2f} -> {(e - c0) / 1e3:9.2f}  ({(e - s) / 1e3:7.2f}){gap}")
            if k == "ens":
                prev_end = e




def blocks(path, block=20):
    """per block of `block` consecutive ensemble launches in the longest cluster: mean launch duration, mean idle gap
    before a launch, launches that started > 10 us after the previous one ended, and the slot / bucket durations"""
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            if k:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    ens = [r for r in rows if r[2] == "ens"]
    clusters, cur = [], [ens[0]]
    for a, b in zip(ens, ens[1:]):
        if b[0] - a[1] > 2_000_000:
            clusters.append(cur)
            cur = []
        cur.append(b)
    clusters.append(cur)
    for c in clusters:
        if len(c) >= 5 * block:
            _blocks(rows, c, block)


def _blocks(rows, c, block):
    print(f"cluster: {len(c)} ensemble launches; per block of {block}:")
    print("  block  us/step  ens_us  gap_us  late(>10us)  slot_us  lean_us")
    for b0 in range(0, len(c) - block + 1, block):
        blk = c[b0:b0 + block]
        lo, hi = blk[0][0], blk[-1][1]
        dur = [(e - s) / 1e3 for s, e, _ in blk]
        gaps = [(y[0] - x[1]) / 1e3 for x, y in zip(blk, blk[1:])]
        sl = [(e - s) / 1e3 for s, e, k in rows if k == "slot" and lo <= s <= hi]
        ln = [(e - s) / 1e3 for s, e, k in rows if k == "lean" and lo <= s <= hi]
        print(f"  {b0 // block:5d}  {(hi - lo) / 1e3 / block:7.2f}  {sum(dur) / len(dur):6.2f}  "
              f"{sum(gaps) / len(gaps):6.2f}  {sum(g > 10 for g in gaps):11d}  "
              f"{sum(sl) / max(1, len(sl)):7.2f}  {sum(ln) / max(1, len(ln)):7.2f}")


def dump(path, out):
    """the step kernels only (start, end, kind), a compact copy of the trace for offline analysis"""
    with open(path) as f, open(out, "w") as o:
        o.write("Start_Timestamp,End_Timestamp,Kernel_Name\n")
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            if k:
                o.write(f"{r['Start_Timestamp']},{r['End_Timestamp']},{k}\n")


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[2] == "dump":
        dump(sys.argv[1], sys.argv[3])
    elif len(sys.argv) > 2 and sys.argv[2] == "blocks":
        blocks(sys.argv[1])
    else:
        main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
