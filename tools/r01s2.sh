cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/s2.pytest.log 2>&1; rc=$?; echo rc=$rc; tail -40 gpurun_out/s2.pytest.log
exit $rc
