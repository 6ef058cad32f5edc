#!/bin/bash
# config 4: issue priorities of the pipelined stream's kernels (the fused kernel at 0 by default now): the lean
# bucket kernel at priority 2 (feature_prio 1) against 0
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-fprio}
for V in 1 0 1; do
  timeout -k 10 300 python -u bench.py --workload config4 --no-cpu-baseline --steps 400 --engine-option feature_prio=$V > gpurun_out/$T.$V.log 2>&1 || { tail -20 gpurun_out/$T.$V.log; exit 1; }
  grep '^{' gpurun_out/$T.$V.log > gpurun_out/$T.$V.json
  python3 -c "import json; d=json.load(open('gpurun_out/$T.$V.json')); p=d['parity_vs_oracle']; print('fprio=$V', d['value'], d['ms_per_step'], d['kernel_avg_us'], {k: p.get(k) for k in ('vector_mismatched_elements','max_abs_prob_diff','decision_mismatches')})"
done
