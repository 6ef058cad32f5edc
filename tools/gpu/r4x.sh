#!/bin/bash
# round 4: config 3j, the scoring engine's ensemble chunk layout (compact: room for a codec workgroup on the CU)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4x}
for V in "--engine-option ensemble_chunks=2" "" "--engine-option ensemble_chunks=2"; do
  N=$(echo "x$V" | tr -d ' -=')
  timeout -k 10 300 python -u bench.py --workload config3j --no-cpu-baseline $V > gpurun_out/$T.$N.log 2>&1 || { tail -20 gpurun_out/$T.$N.log; exit 1; }
  grep '^{' gpurun_out/$T.$N.log > gpurun_out/$T.$N.json
  python3 -c "import json; d=json.load(open('gpurun_out/$T.$N.json')); print('$V', d['value'], d['ms_per_step'], d['kernel_avg_us'], d['parity_vs_oracle']['decision_mismatches'])"
done
