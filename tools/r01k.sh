cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r01k.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -5 gpurun_out/r01k.pytest.log
[ $rc -ne 0 ] && exit $rc
VARIANTS=1,2 timeout -k 10 300 python tools/forest_sweep.py > gpurun_out/r01k.sweep.log 2>&1; rc=$?; echo sweep_rc=$rc; cat gpurun_out/r01k.sweep.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 100 --warmup 10 > gpurun_out/r01k.bench2.log 2>&1; rc=$?; echo bench2_rc=$rc; tail -2 gpurun_out/r01k.bench2.log
exit $rc
