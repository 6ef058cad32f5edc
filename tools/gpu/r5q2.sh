#!/bin/bash
# the driver command's short region: per-block rates after it (FD_BENCH_BLOCKS), then with a long warm-up, then the
# default line under a kernel trace (timeline of the timed region kept for tools/trace_steps.py)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q2}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], d['host_submit_ms_per_step'], (d.get('host_submit_breakdown') or {}).get('native_us_per_step'), d.get('diag_blocks_ms_per_step'))" "$1"; }
B="--no-cpu-baseline --latency-iters 0 --loaded-iters 0 --alone-iters 0"
FD_BENCH_BLOCKS=8 timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 $B > gpurun_out/$T.a.json 2> gpurun_out/$T.a.log || { tail -20 gpurun_out/$T.a.log; exit 1; }
summ gpurun_out/$T.a.json
FD_BENCH_BLOCKS=4 timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 200 $B > gpurun_out/$T.b.json 2> gpurun_out/$T.b.log || { tail -20 gpurun_out/$T.b.log; exit 1; }
summ gpurun_out/$T.b.json
FD_BENCH_BLOCKS=4 timeout -k 10 400 python3 -u bench.py --steps 200 --warmup 5 $B > gpurun_out/$T.c.json 2> gpurun_out/$T.c.log || { tail -20 gpurun_out/$T.c.log; exit 1; }
summ gpurun_out/$T.c.json
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/$T.tr -o run -- python3 -u bench.py --steps 20 --warmup 5 $B > gpurun_out/$T.tr.log 2>&1 || { tail -20 gpurun_out/$T.tr.log; exit 1; }
f=$(find /tmp/$T.tr -name '*kernel_trace.csv' | head -1)
python3 tools/trace_steps.py "$f" > gpurun_out/$T.timeline.txt || exit 1
tail -60 gpurun_out/$T.timeline.txt
