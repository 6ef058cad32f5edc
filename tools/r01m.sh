cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_forest.py -m gpu -x -q > gpurun_out/r01m.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/r01m.pytest.log
[ $rc -ne 0 ] && exit $rc
VARIANTS=1,2 timeout -k 10 300 python tools/forest_sweep.py > gpurun_out/r01m.sweep.log 2>&1; rc=$?; echo sweep_rc=$rc; tail -3 gpurun_out/r01m.sweep.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/forest_phases.py > gpurun_out/r01m.phases.log 2>&1; rc=$?; echo phases_rc=$rc; tail -9 gpurun_out/r01m.phases.log
exit $rc
