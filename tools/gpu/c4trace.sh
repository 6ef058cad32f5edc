#!/bin/bash
# config 4 pipelined stream: kernel trace -> the ensemble-to-ensemble idle time and what runs in it
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-c4trace}; shift
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T -o trace -- python3 -u bench.py --workload config4 --no-cpu-baseline --steps 200 --latency-iters 10 --loaded-iters 10 --alone-iters 5 --timing-steps 20 "$@" > gpurun_out/$T.log 2>&1 || { tail -20 gpurun_out/$T.log; exit 1; }
F=$(find gpurun_out/$T -name "*kernel_trace.csv"); python3 tools/pipe_gaps.py $F > gpurun_out/$T.gaps.txt && python3 tools/pipe_gaps.py $F timeline > gpurun_out/$T.timeline.txt && cat gpurun_out/$T.gaps.txt
rm -f $(find gpurun_out/$T -name '*kernel_trace.csv')
