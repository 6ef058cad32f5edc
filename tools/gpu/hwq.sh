#!/bin/bash
# hardware queues per process (HIP's GPU_MAX_HW_QUEUES, default 4) vs the native sharded step and the direct step
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q}
for Q in 4 8 12; do
  echo "== GPU_MAX_HW_QUEUES=$Q" >> gpurun_out/$T.hwq.log
  GPU_MAX_HW_QUEUES=$Q VARIANTS=direct,native timeout -k 10 300 python -u tools/route_overhead.py >> gpurun_out/$T.hwq.log 2>&1 || exit $?
done
for Q in 4 8; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 400 python -u bench.py --steps 200 --warmup 20 > gpurun_out/$T.bench_q$Q.json 2> gpurun_out/$T.bench_q$Q.err || exit $?
done
export GPU_MAX_HW_QUEUES=8
VARIANTS=native STEPS=60 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/$T.prof -o run -- \
  python tools/route_overhead.py > gpurun_out/$T.prof.log 2>&1 || exit $?
t=$(find /tmp/$T.prof -name '*kernel_trace.csv' | head -1)
TRACE_SKIP=30 python tools/trace_gaps.py "$t" 60 ensemble feat_slot feat_bucket pipe_out route nccl Nccl scatter result > gpurun_out/$T.trace_gaps.txt 2>&1
rm -rf /tmp/$T.prof
