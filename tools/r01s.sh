cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_lstm.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r01s.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -25 gpurun_out/r01s.pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --workload config5 --steps 200 --warmup 20 --latency-iters 300 --cpu-seconds 8 > gpurun_out/r01s.c5.log 2>&1; rc=$?; echo c5_rc=$rc; tail -3 gpurun_out/r01s.c5.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01s.c5prof -o run -- python bench.py --workload config5 --steps 100 --warmup 5 --latency-iters 5 --no-cpu-baseline > gpurun_out/r01s.c5prof.log 2>&1; rc=$?; echo c5prof_rc=$rc
exit $rc
