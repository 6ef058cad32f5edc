cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fmap.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r01y.fmap.log 2>&1; rc=$?; echo fmap_rc=$rc; tail -30 gpurun_out/r01y.fmap.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r01y.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/r01y.pytest.log
exit $rc
