#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-o}
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharding.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$T.pytest.log; [ $rc -ne 0 ] && exit $rc
VARIANTS=direct,native timeout -k 10 400 python -u tools/route_overhead.py > gpurun_out/$T.route_overhead.log 2>&1 || exit $?
bash tools/gpu/trace_native.sh $T
