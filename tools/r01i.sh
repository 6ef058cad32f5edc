cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r01i.pytest.log 2>&1; echo pytest_rc=$?; tail -2 gpurun_out/r01i.pytest.log
timeout -k 10 600 python bench.py --steps 200 --warmup 20 > gpurun_out/r01i.bench2.log 2>&1; rc=$?; echo bench2_rc=$rc; tail -1 gpurun_out/r01i.bench2.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py --workload config3 --steps 100 --warmup 10 --latency-iters 50 > gpurun_out/r01i.bench3.log 2>&1; rc=$?; echo bench3_rc=$rc; tail -3 gpurun_out/r01i.bench3.log
