#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-l}
timeout -k 10 400 python -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_latency.py -m gpu -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -2 gpurun_out/$T.pytest.log
WORKLOADS=config5 bash tools/gpu/workloads.sh $T || exit 1
WORKLOADS=5 bash tools/gpu/pmc_r03.sh $T || exit 1
