#!/bin/bash
# kernel traces of the driver's command with 8 diagnostic blocks after the timed region, latency loops after (0) and
# before (1) it: per-block ensemble duration / idle gaps / late launches (tools/trace_steps.py blocks)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q5}
for k in 0 1; do
  FD_BENCH_LATENCY_FIRST=$k FD_BENCH_BLOCKS=8 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/$T.tr$k -o run -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --loaded-iters 0 --alone-iters 0 > gpurun_out/$T.tr$k.log 2>&1 || { tail -20 gpurun_out/$T.tr$k.log; exit 1; }
  f=$(find /tmp/$T.tr$k -name '*kernel_trace.csv' | head -1)
  echo "latency first = $k"; grep '^{' gpurun_out/$T.tr$k.log | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d.get('diag_blocks_ms_per_step'))"
  python3 tools/trace_steps.py "$f" dump gpurun_out/$T.steps$k.csv && python3 tools/trace_steps.py gpurun_out/$T.steps$k.csv blocks | tee gpurun_out/$T.blocks$k.txt
done
