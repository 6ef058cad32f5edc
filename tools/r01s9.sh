cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/s9.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -30 gpurun_out/s9.pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ingest_ua_exp.py > gpurun_out/s9.time.log 2>&1; rc=$?; echo time_rc=$rc; cat gpurun_out/s9.time.log | grep stop
exit $rc
