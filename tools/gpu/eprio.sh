#!/bin/bash
# config 4: the fused kernel's issue priority over the co-running feature kernels (ensemble_prio 1 = s_setprio 2)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-eprio}
for V in 0 1 0; do
  timeout -k 10 300 python -u bench.py --workload config4 --no-cpu-baseline --steps 400 --engine-option ensemble_prio=$V > gpurun_out/$T.$V.log 2>&1 || { tail -20 gpurun_out/$T.$V.log; exit 1; }
  grep '^{' gpurun_out/$T.$V.log > gpurun_out/$T.$V.json
  python3 -c "import json; d=json.load(open('gpurun_out/$T.$V.json')); p=d['parity_vs_oracle']; print('prio=$V', d['value'], d['ms_per_step'], d['kernel_avg_us'], {k: p.get(k) for k in ('vector_mismatched_elements','max_abs_prob_diff','decision_mismatches')})"
done
