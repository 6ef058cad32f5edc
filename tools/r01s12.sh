#!/bin/bash
# forest kernel A/B (VARIANTS = forest_kernel options): GPU forest parity tests, interleaved XGB + IF sweeps, bench
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s12}
timeout -k 10 600 python -u -m pytest tests/test_gpu_forest.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/$T.pytest.log
[ $rc -ne 0 ] && exit $rc
VARIANTS=${VARIANTS:-3,7} timeout -k 10 300 python tools/forest_sweep.py > gpurun_out/$T.sweep.log 2>&1; rc=$?; echo sweep_rc=$rc; tail -3 gpurun_out/$T.sweep.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --latency-iters 50 > gpurun_out/$T.bench.log 2>&1; rc=$?; echo bench_rc=$rc; grep -o '"kernel_avg_us": [0-9.]*' gpurun_out/$T.bench.log; grep -o '"value": [0-9.]*' gpurun_out/$T.bench.log

[ $rc -ne 0 ] && exit $rc
IF=1 VARIANTS=${VARIANTS:-3,7} timeout -k 10 300 python tools/forest_sweep.py > gpurun_out/$T.sweep_if.log 2>&1; rc=$?; echo sweep_if_rc=$rc; tail -3 gpurun_out/$T.sweep_if.log
exit $rc
