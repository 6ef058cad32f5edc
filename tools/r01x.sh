cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r01x.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -4 gpurun_out/r01x.pytest.log
[ $rc -ne 0 ] && exit $rc
for B in 1024 16384; do VARIANTS=3,6 B=$B timeout -k 10 300 python tools/forest_sweep.py > gpurun_out/r01x.sweep$B.log 2>&1; rc=$?; echo sweep${B}_rc=$rc; tail -2 gpurun_out/r01x.sweep$B.log; [ $rc -ne 0 ] && exit $rc; done
timeout -k 10 600 python bench.py --workload config5 --steps 200 --warmup 20 --latency-iters 300 --cpu-seconds 5 > gpurun_out/r01x.c5.log 2>&1; rc=$?; echo c5_rc=$rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01x.c5prof -o run -- python bench.py --workload config5 --steps 100 --warmup 5 --latency-iters 20 --no-cpu-baseline > gpurun_out/r01x.c5prof.log 2>&1; rc=$?; echo c5prof_rc=$rc
exit $rc
