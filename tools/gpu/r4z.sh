#!/bin/bash
# round 4: the ensemble kernel's two-level binning (option ensemble_bin_index) A/B, config 4 and config 2, parity in line
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4z}
for W in config4 config2; do
  for V in 0 1; do
    timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline --engine-option ensemble_bin_index=$V > gpurun_out/$T.$W.$V.log 2>&1 || { tail -20 gpurun_out/$T.$W.$V.log; exit 1; }
    grep '^{' gpurun_out/$T.$W.$V.log > gpurun_out/$T.$W.$V.json
    python3 -c "import json; d=json.load(open('gpurun_out/$T.$W.$V.json')); p=d['parity_vs_oracle']; print('$W idx=$V', d['value'], d['ms_per_step'], d['kernel_avg_us'], d.get('kernel_avg_us_alone'), {k: p.get(k) for k in ('vector_mismatched_elements','max_abs_prob_diff','decision_mismatches','max_abs_model_prob_diff')})"
  done
done
