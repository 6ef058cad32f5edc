cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r01z.smoke.log 2>&1; rc=$?; echo smoke_rc=$rc; tail -2 gpurun_out/r01z.smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r01z.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/r01z.pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r01z.bench.log 2>&1; rc=$?; echo bench_rc=$rc; tail -1 gpurun_out/r01z.bench.log
exit $rc
