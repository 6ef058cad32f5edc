cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_forest.py tests/test_gpu_lstm.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r01w.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -4 gpurun_out/r01w.pytest.log
[ $rc -ne 0 ] && exit $rc
for B in 1024 4096 16384 32768; do VARIANTS=3,6 B=$B timeout -k 10 300 python tools/forest_sweep.py > gpurun_out/r01w.sweep$B.log 2>&1; rc=$?; echo sweep${B}_rc=$rc; tail -2 gpurun_out/r01w.sweep$B.log; [ $rc -ne 0 ] && exit $rc; done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01w.c5prof -o run -- python bench.py --workload config5 --steps 100 --warmup 5 --latency-iters 20 --no-cpu-baseline > gpurun_out/r01w.c5prof.log 2>&1; rc=$?; echo c5prof_rc=$rc; grep '^{' gpurun_out/r01w.c5prof.log | cut -c1-300
exit $rc
