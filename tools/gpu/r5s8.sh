#!/bin/bash
# rocprofv3 kernel-trace stats of the driver's command (secondaries off); the trace itself is dropped on the box so
# the call's gpurun_out stays small (the stats csv comes back)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s8}
FD_BENCH_SECONDARY=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$T.prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$T.prof_bench.json 2> gpurun_out/$T.prof.log || { tail -20 gpurun_out/$T.prof.log; exit 1; }
f=$(find /tmp/$T.prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/$T.prof_kernel_stats.csv
python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r['Name'] for k in ('ensemble_kernel','feat_slot','feat_bucket_lean')): print(r['Name'][:60], r['Calls'], r['AverageNs'])
" gpurun_out/$T.prof_kernel_stats.csv
