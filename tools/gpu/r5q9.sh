#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q9}
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_configs.py tests/test_gpu_features_segments.py -x -v --timeout 300 --timeout-method thread > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
bash tools/gpu/ab5.sh $T "--engine-option split_sort=0" "--engine-option split_sort=1"
