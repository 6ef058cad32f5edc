#!/bin/bash
# config 3 (10 M cards): the slot pass on its own stream (slot_stream 2, config 4's auto choice) against the auto
# choice at 2^24 slots (0), alternating, two rounds
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6t}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d.get('kernel_avg_us'); print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], k, (d.get('parity_vs_oracle') or {}).get('timed_path', {}).get('max_abs_prob_diff'))" "$1"; }
X="--workload config3 --no-cpu-baseline --loaded-iters 0 --alone-iters 0 --latency-iters 0"
for r in 1 2; do
  for v in 0 2; do
    timeout -k 10 300 python3 -u bench.py $X --engine-option slot_stream=$v > gpurun_out/$T.s$v.$r.json 2> gpurun_out/$T.s$v.$r.log || { tail -5 gpurun_out/$T.s$v.$r.log; exit 1; }
    echo "[slot_stream=$v]"; summ gpurun_out/$T.s$v.$r.json
  done
done
