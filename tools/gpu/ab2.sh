#!/bin/bash
# ab.sh plus a kernel trace of the default bench (stats kept, the raw trace reduced on the box)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; shift
bash tools/gpu/ab.sh "$@" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$T.prof -o run -- \
  python bench.py --no-cpu-baseline --steps 100 --warmup 5 --latency-iters 0 --loaded-iters 0 --alone-iters 20 > gpurun_out/$T.prof.log 2>&1 || exit $?
f=$(find /tmp/$T.prof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/$T.kernel_stats.csv
t=$(find /tmp/$T.prof -name '*kernel_trace.csv' | head -1)
TRACE_SKIP=120 python tools/trace_gaps.py "$t" 60 ensemble feat_slot feat_bucket pipe_out > gpurun_out/$T.trace_gaps.txt 2>&1
rm -rf /tmp/$T.prof
