"""Kernel timeline of a rocprofv3 --kernel-trace run: per kernel start/end/duration/queue and the idle gap on
the queue of the dominant kernel (usage: python tools/trace_gaps.py run_kernel_trace.csv [n] [names...])."""
import csv
import os
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
names = sys.argv[3:] or ["ensemble", "feat_slot", "feat_bucket"]
rows = list(csv.DictReader(open(path)))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows)
sel = [k for k in ks if any(x in k[2] for x in names)]
skip = int(os.environ.get("TRACE_SKIP", "20"))  # kernels at the end left out (e.g. the bench's alone / latency loops)
win = sel[-(n + skip):-skip] if len(sel) > n + skip else sel
t0 = win[0][0]
last_end = {}
for s, e, name, q in win:
    nm = name.replace("void ", "").replace("fd::(anonymous namespace)::", "")[:32]
    gap = (s - last_end[q]) / 1000 if q in last_end else 0.0
    last_end[q] = e
    print(f"{(s - t0) / 1000:9.1f} {(e - t0) / 1000:9.1f} {(e - s) / 1000:7.1f}  qgap {gap:6.1f}  q{q} {nm}")

# resources of each distinct kernel in the window (what co-residence with the fused kernel depends on)
seen = {}
for r in rows:
    nm = r["Kernel_Name"].replace("void ", "").replace("fd::(anonymous namespace)::", "")[:40]
    if nm in seen or not any(x in r["Kernel_Name"] for x in names):
        continue
    seen[nm] = {c: r[c] for c in r if any(t in c.lower() for t in ("lds", "vgpr", "sgpr", "workgroup", "grid",
                                                                   "scratch", "accum"))}
for nm, v in seen.items():
    print(f"{nm:40s} {v}")

