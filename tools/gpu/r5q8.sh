#!/bin/bash
# the ramp over the first ~150 pipelined steps: is it the slot stream, the pipeline, or below the engine?
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q8}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], d.get('diag_blocks_ms_per_step'))" "$1"; }
B="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --loaded-iters 0 --alone-iters 0 --latency-iters 0"
k=0
for args in "" "--engine-option slot_stream=0" "--no-pipeline" "--engine-option feature_prio=1"; do
  k=$((k + 1))
  FD_BENCH_LATENCY_FIRST=0 FD_BENCH_BLOCKS=10 timeout -k 10 400 python3 -u bench.py $B $args > gpurun_out/$T.$k.json 2> gpurun_out/$T.$k.log || { tail -5 gpurun_out/$T.$k.log; exit 1; }
  echo "$args"; summ gpurun_out/$T.$k.json
done
