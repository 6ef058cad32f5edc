cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python tools/ingest_phases.py > gpurun_out/s5.phases.log 2>&1; rc=$?; echo phases_rc=$rc; cat gpurun_out/s5.phases.log | grep stop_after
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/s5.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/s5.pytest.log
exit $rc
