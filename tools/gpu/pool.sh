#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-j}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ensemble.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$T.pytest.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --loaded-iters 200 --ensemble-pool $v > gpurun_out/$T.b$v.log 2>&1 || exit $?
grep '^{' gpurun_out/$T.b$v.log > gpurun_out/$T.b$v.json
POOL=$v timeout -k 10 300 python -u tools/ens_phases_pipe.py > gpurun_out/$T.phases$v.log 2>&1 || exit $?
done
