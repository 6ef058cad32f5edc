#!/bin/bash
# round 4 (slot stream): the whole -m gpu suite, then config 4 default / slot_stream 0, config 3j, config 3
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r5b}
bash tools/gpu/r4b.sh $T || exit $?
B="--no-cpu-baseline --steps 400 --latency-iters 0 --loaded-iters 0"
for args in "" "--engine-option slot_stream=0" "--workload config3j" "--workload config3j --engine-option slot_stream=0" "--workload config3"; do
  k=$((k + 1))
  timeout -k 10 400 python -u bench.py $B $args > gpurun_out/$T.b$k.log 2>&1 || { tail -20 gpurun_out/$T.b$k.log; exit 1; }
  grep '^{' gpurun_out/$T.b$k.log > gpurun_out/$T.b$k.json
  python3 -c "import json; d=json.load(open('gpurun_out/$T.b$k.json')); print('$args', d['value']/1e6, d['ms_per_step'], d['kernel_avg_us'], d.get('parity_vs_oracle'))"
done
