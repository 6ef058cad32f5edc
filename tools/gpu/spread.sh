#!/bin/bash
# bucket_spread A/B: feature/latency GPU tests with the default (1), then config 5 and config 4 at 0 and 1
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-spread}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_latency.py tests/test_gpu_features.py tests/test_gpu_configs.py -k "latency or config5 or small or fused or lstm or features" > gpurun_out/$T.tests.log 2>&1 || { tail -30 gpurun_out/$T.tests.log; exit 1; }
tail -2 gpurun_out/$T.tests.log
for W in config5 config4; do
  for V in 0 1; do
    timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline --engine-option bucket_spread=$V > gpurun_out/$T.$W.$V.log 2>&1 || { tail -20 gpurun_out/$T.$W.$V.log; exit 1; }
    grep '^{' gpurun_out/$T.$W.$V.log > gpurun_out/$T.$W.$V.json
    python3 -c "import json; d=json.load(open('gpurun_out/$T.$W.$V.json')); p=d['parity_vs_oracle']; print('$W spread=$V', d['value'], d['ms_per_step'], d['kernel_avg_us'], {k: p.get(k) for k in ('vector_mismatched_elements','max_abs_prob_diff','decision_mismatches')})"
  done
done
