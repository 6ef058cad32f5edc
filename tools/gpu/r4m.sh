#!/bin/bash
# round 4: A/B of the ensemble kernel's level-based walk priority (option ensemble_dyn_prio), config 4 and config 2
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4m}
for V in 0 1; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --engine-option ensemble_dyn_prio=$V > gpurun_out/$T.c4_p$V.log 2>&1 || exit $?
  grep '^{' gpurun_out/$T.c4_p$V.log > gpurun_out/$T.c4_p$V.json
  python3 -c "import json; d=json.load(open('gpurun_out/$T.c4_p$V.json')); print('c4 dyn=$V', d['value'], d['ms_per_step'], d['kernel_avg_us'], d['kernel_avg_us_alone'])"
done
for V in 0 1; do
  timeout -k 10 300 python -u bench.py --workload config2 --no-cpu-baseline --engine-option ensemble_dyn_prio=$V > gpurun_out/$T.c2_p$V.log 2>&1 || exit $?
  grep '^{' gpurun_out/$T.c2_p$V.log > gpurun_out/$T.c2_p$V.json
  python3 -c "import json; d=json.load(open('gpurun_out/$T.c2_p$V.json')); print('c2 dyn=$V', d['value'], d['ms_per_step'], d['kernel_avg_us'])"
done
