#!/bin/bash
# round 4: config 5 through the pipelined stream vs one call per step; small_streams variants
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4o}
for V in "" "--pipeline" "--pipeline --small-streams 1" "--small-streams 1"; do
  N=$(echo "x$V" | tr -d ' -')
  timeout -k 10 200 python -u bench.py --workload config5 --no-cpu-baseline $V > gpurun_out/$T.$N.log 2>&1 || exit $?
  grep '^{' gpurun_out/$T.$N.log > gpurun_out/$T.$N.json
  python3 -c "import json; d=json.load(open('gpurun_out/$T.$N.json')); print('$V', d['value'], d['ms_per_step'], d['p99_batch_latency_ms'], d['kernel_avg_us'], d['parity_vs_oracle'].get('decision_mismatches'))"
done
