#!/bin/bash
# pipelined stream: output-staging wait placement A/B (config 4, then config 3j), parity in line
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-cwait}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipeline.py > gpurun_out/$T.tests.log 2>&1 || { tail -30 gpurun_out/$T.tests.log; exit 1; }
tail -1 gpurun_out/$T.tests.log
for W in config4; do
  for V in 0 1; do
    timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline --engine-option pipe_copy_query=$V > gpurun_out/$T.$W.$V.log 2>&1 || { tail -20 gpurun_out/$T.$W.$V.log; exit 1; }
    grep '^{' gpurun_out/$T.$W.$V.log > gpurun_out/$T.$W.$V.json
    python3 -c "import json; d=json.load(open('gpurun_out/$T.$W.$V.json')); p=d['parity_vs_oracle']; print('$W query=$V', d['value'], d['ms_per_step'], d['kernel_avg_us'], {k: p.get(k) for k in ('vector_mismatched_elements','max_abs_prob_diff','decision_mismatches')})"
  done
done
