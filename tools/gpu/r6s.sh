#!/bin/bash
# kernel trace of 200 pipelined config-4 steps on the current tree: per-step slot / lean / ensemble timing
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6s}
export FD_BENCH_SECONDARY=0
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/$T.tr -o run -- python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --loaded-iters 0 --alone-iters 0 --latency-iters 0 --timing-steps 0 > gpurun_out/$T.tr.log 2>&1 || { tail -20 gpurun_out/$T.tr.log; exit 1; }
f=$(find /tmp/$T.tr -name '*kernel_trace.csv' | head -1)
grep '^{' gpurun_out/$T.tr.log | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'])"
python3 tools/trace_steps.py "$f" dump gpurun_out/$T.steps.csv && python3 tools/trace_steps.py gpurun_out/$T.steps.csv blocks | tee gpurun_out/$T.blocks.txt
