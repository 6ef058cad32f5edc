#!/bin/bash
# eight output staging slots: pipeline tests, then config 4 and config 3 lines
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-pout}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_configs.py tests/test_gpu_sharding_loopback.py > gpurun_out/$T.tests.log 2>&1 || { tail -30 gpurun_out/$T.tests.log; exit 1; }
tail -1 gpurun_out/$T.tests.log
for W in config4 config3; do
  timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline > gpurun_out/$T.$W.log 2>&1 || { tail -20 gpurun_out/$T.$W.log; exit 1; }
  grep '^{' gpurun_out/$T.$W.log > gpurun_out/$T.$W.json
  python3 -c "import json; d=json.load(open('gpurun_out/$T.$W.json')); p=d['parity_vs_oracle']; print('$W', d['value'], d['ms_per_step'], d['kernel_avg_us'], d['p99_batch_latency_ms'], d['loaded_latency']['p99_ms'], {k: p.get(k) for k in ('vector_mismatched_elements','max_abs_prob_diff','decision_mismatches')})"
done
