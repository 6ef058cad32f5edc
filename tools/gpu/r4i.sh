#!/bin/bash
# round 4: card pages (header + ring in one page per slot): parity tests of every card-state user, config 4 bench,
# load-factor comparison, rocprof kernel stats
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4i}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_features.py tests/test_gpu_features_segments.py tests/test_gpu_snapshot.py tests/test_gpu_windows.py \
  tests/test_gpu_pipeline.py tests/test_gpu_configs.py tests/test_gpu_sharding_loopback.py \
  > gpurun_out/$T.pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$T.pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/$T.bench.log 2>&1 || exit $?
grep '^{' gpurun_out/$T.bench.log > gpurun_out/$T.bench.json
python3 -c "import json; d=json.load(open('gpurun_out/$T.bench.json')); print(d['value'], d['ms_per_step'], d['kernel_avg_us'], d['kernel_avg_us_alone'])"
bash tools/gpu/r4h.sh $T
