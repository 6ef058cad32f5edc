#!/bin/bash
# loaded-latency diagnosis: bench (no CPU baseline) then a kernel trace of the same run
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-b}
timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-iters 50 --loaded-iters 400 > gpurun_out/$T.bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T.prof -o run -- \
  python bench.py --no-cpu-baseline --steps 50 --warmup 5 --latency-iters 10 --loaded-iters 400 > gpurun_out/$T.prof.log 2>&1
