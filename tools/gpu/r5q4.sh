#!/bin/bash
# A/B in one call: the driver's command with the latency loops before (1) / after (0) the throughput region, with
# 8 blocks of 20 steps after the timed region; then a 400-step line (the box's steady state)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q4}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], d['host_submit_ms_per_step'], (d.get('host_submit_breakdown') or {}).get('native_us_per_step'), d.get('diag_blocks_ms_per_step'))" "$1"; }
for k in 0 1 0 1; do
  j=$((j + 1))
  FD_BENCH_LATENCY_FIRST=$k FD_BENCH_BLOCKS=8 timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --loaded-iters 0 --alone-iters 0 > gpurun_out/$T.l$k.$j.json 2> gpurun_out/$T.l$k.$j.log || { tail -20 gpurun_out/$T.l$k.$j.log; exit 1; }
  summ gpurun_out/$T.l$k.$j.json
done
timeout -k 10 400 python3 -u bench.py --steps 400 --no-cpu-baseline --loaded-iters 0 --alone-iters 0 > gpurun_out/$T.s400.json 2> gpurun_out/$T.s400.log || { tail -20 gpurun_out/$T.s400.log; exit 1; }
summ gpurun_out/$T.s400.json
