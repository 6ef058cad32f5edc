cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/s4.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/s4.pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --workload ingest --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/s4.ingest.log 2>&1; rc=$?; echo ingest_rc=$rc; tail -1 gpurun_out/s4.ingest.log | cut -c1-900
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py --workload config3j --steps 100 --warmup 10 --cpu-seconds 8 --latency-iters 100 > gpurun_out/s4.c3j.log 2>&1; rc=$?; echo c3j_rc=$rc; tail -2 gpurun_out/s4.c3j.log
exit $rc
