#!/bin/bash
# split-row ring fix: the pipelined twin tests (every slot-stream form), features, configs, loopback, latency
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6l}
timeout -k 10 1100 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_features.py tests/test_gpu_features_segments.py tests/test_gpu_configs.py tests/test_gpu_latency.py tests/test_gpu_sharding_loopback.py -v --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/$T.pytest.log | grep -v PASSED | head -20; tail -1 gpurun_out/$T.pytest.log; exit $rc
