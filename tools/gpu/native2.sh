#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-m}
timeout -k 10 150 python -u -m pytest tests/test_gpu_sharding_mp.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k native > gpurun_out/$T.native2.log 2>&1; rc=$?; tail -5 gpurun_out/$T.native2.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python -u tools/route_overhead.py > gpurun_out/$T.route_overhead.log 2>&1 || exit $?
