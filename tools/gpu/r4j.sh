#!/bin/bash
# round 4: ensemble kernel back to 62 VGPRs (compact prologue in the row's registers) + card pages: parity, config 4
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4j}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ensemble.py tests/test_gpu_pipeline.py tests/test_gpu_latency.py tests/test_gpu_configs.py \
  > gpurun_out/$T.pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$T.pytest.log; [ $rc -ne 0 ] && exit $rc
for V in "" "--ring-k 16 --slots-per-card 1.6"; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $V > gpurun_out/$T.bench.log 2>&1 || exit $?
  grep '^{' gpurun_out/$T.bench.log > gpurun_out/$T.bench$(echo $V | tr -d ' -.').json
  python3 -c "import json; d=json.load(open('gpurun_out/$T.bench$(echo $V | tr -d ' -.').json')); print('$V', d['value'], d['ms_per_step'], d['kernel_avg_us'], d['kernel_avg_us_alone'])"
done
