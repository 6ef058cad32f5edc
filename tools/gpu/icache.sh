#!/bin/bash
# instruction-cache counters of the ingest kernel (one rocprofv3 --pmc pass under a hard limit)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-ic}
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_VALU SQ_WAVES --output-format csv -d /tmp/$T.p -o run -- \
  python bench.py --workload ingest --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 2 --loaded-iters 0 --alone-iters 2 --parity-batches 1 > gpurun_out/$T.log 2>&1
rc=$?; echo "rc=$rc"
f=$(find /tmp/$T.p -name '*counter_collection.csv' | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:60]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k, cs in acc.items():
    d = len(n[k]); print(k, d, {c: round(v / d) for c, v in cs.items()})
PY
rm -rf /tmp/$T.p
exit $rc
