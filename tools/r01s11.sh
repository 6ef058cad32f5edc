#!/bin/bash
# forest kernel A/B: GPU forest parity tests + config2 bench line (no CPU leg)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s11}
timeout -k 10 600 python -u -m pytest tests/test_gpu_forest.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/$T.pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --latency-iters 50 > gpurun_out/$T.bench.log 2>&1; rc=$?; echo bench_rc=$rc; tail -1 gpurun_out/$T.bench.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --latency-iters 50 --workload config3 > gpurun_out/$T.bench3.log 2>&1; rc=$?; echo bench3_rc=$rc; tail -1 gpurun_out/$T.bench3.log | cut -c1-300
exit $rc
