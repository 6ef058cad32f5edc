#!/bin/bash
# config 5 (1 k latency batches): kernel trace of back-to-back steps -> per-kernel duration and the gap before it
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-c5trace}; shift
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T -o trace -- python3 -u bench.py --workload config5 --no-cpu-baseline --steps 400 --latency-iters 20 --loaded-iters 20 --alone-iters 5 "$@" > gpurun_out/$T.log 2>&1 || { tail -20 gpurun_out/$T.log; exit 1; }
grep '^{' gpurun_out/$T.log > gpurun_out/$T.json
python3 tools/kernel_gaps.py $(find gpurun_out/$T -name '*kernel_trace.csv') > gpurun_out/$T.gaps.txt && cat gpurun_out/$T.gaps.txt
