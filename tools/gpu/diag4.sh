#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-i}
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$T.pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ens_phases_pipe.py > gpurun_out/$T.ens_phases_pipe.log 2>&1 || exit $?
FD_STALL_TRACE=3 timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-iters 100 --loaded-iters 400 > gpurun_out/$T.stall.log 2>&1 || exit $?
