#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_features_segments.py tests/test_gpu_latency.py tests/test_gpu_configs.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -2 gpurun_out/$T.pytest.log
WORKLOADS="config5" bash tools/gpu/workloads.sh $T || exit 1
