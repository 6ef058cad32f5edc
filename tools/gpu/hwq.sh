#!/bin/bash
# hardware queues per process (HIP's GPU_MAX_HW_QUEUES, default 4) vs the native sharded step and the direct step
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q}
for Q in ${QUEUES:-4 5 6 8}; do
  echo "== GPU_MAX_HW_QUEUES=$Q" >> gpurun_out/$T.hwq.log
  GPU_MAX_HW_QUEUES=$Q VARIANTS=${VARIANTS:-direct,native} timeout -k 10 300 python -u tools/route_overhead.py >> gpurun_out/$T.hwq.log 2>&1 || exit $?
done
