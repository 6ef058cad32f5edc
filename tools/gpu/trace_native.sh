#!/bin/bash
# kernel (+ memory copy) trace of the native sharded step on one GPU (route_overhead VARIANTS, default native)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-n}
VARIANTS=${VARIANTS:-native} STEPS=60 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/$T.prof -o run -- \
  python tools/route_overhead.py > gpurun_out/$T.prof.log 2>&1 || exit $?
t=$(find /tmp/$T.prof -name '*kernel_trace.csv' | head -1)
TRACE_SKIP=30 python tools/trace_gaps.py "$t" 80 ensemble feat_slot feat_bucket pipe_out route nccl Nccl scatter result > gpurun_out/$T.trace_gaps.txt 2>&1
m=$(find /tmp/$T.prof -name '*memory_copy_trace.csv' | head -1)
[ -n "$m" ] && tail -n 60 "$m" > gpurun_out/$T.memcpy_tail.csv
rm -rf /tmp/$T.prof
