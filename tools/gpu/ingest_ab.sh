#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-i}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ingest.py -m gpu -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -2 gpurun_out/$T.pytest.log
timeout -k 10 300 python -u tools/ingest_phases.py > gpurun_out/$T.phases.log 2>&1 || exit 1
grep stop_after gpurun_out/$T.phases.log
WORKLOADS="ingest config3j" bash tools/gpu/workloads.sh $T || exit 1
