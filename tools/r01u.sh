cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_forest.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r01u.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -15 gpurun_out/r01u.pytest.log
[ $rc -ne 0 ] && exit $rc
VARIANTS=3,4,5 timeout -k 10 300 python tools/forest_sweep.py > gpurun_out/r01u.sweep.log 2>&1; rc=$?; echo sweep_rc=$rc; tail -4 gpurun_out/r01u.sweep.log
[ $rc -ne 0 ] && exit $rc
VARIANTS=3,4,5 B=1024 timeout -k 10 300 python tools/forest_sweep.py > gpurun_out/r01u.sweep1k.log 2>&1; rc=$?; echo sweep1k_rc=$rc; tail -4 gpurun_out/r01u.sweep1k.log
exit $rc
