#!/bin/bash
# config 4: bucket_keys A/B (keys per bucket workgroup of the feature pass; default 128 at 64 k)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-bkeys}
for V in 64 128 256; do
  timeout -k 10 300 python -u bench.py --workload config4 --no-cpu-baseline --engine-option bucket_keys=$V > gpurun_out/$T.$V.log 2>&1 || { tail -20 gpurun_out/$T.$V.log; exit 1; }
  grep '^{' gpurun_out/$T.$V.log > gpurun_out/$T.$V.json
  python3 -c "import json; d=json.load(open('gpurun_out/$T.$V.json')); p=d['parity_vs_oracle']; print('keys=$V', d['value'], d['ms_per_step'], d['kernel_avg_us'], {k: p.get(k) for k in ('vector_mismatched_elements','max_abs_prob_diff','decision_mismatches')})"
done
