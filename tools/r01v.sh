cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r01v.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -15 gpurun_out/r01v.pytest.log
[ $rc -ne 0 ] && exit $rc
VARIANTS=3,6 B=1024 timeout -k 10 300 python tools/forest_sweep.py > gpurun_out/r01v.sweep1k.log 2>&1; rc=$?; echo sweep1k_rc=$rc; tail -3 gpurun_out/r01v.sweep1k.log
[ $rc -ne 0 ] && exit $rc
VARIANTS=3,6 B=16384 timeout -k 10 300 python tools/forest_sweep.py > gpurun_out/r01v.sweep16k.log 2>&1; rc=$?; echo sweep16k_rc=$rc; tail -3 gpurun_out/r01v.sweep16k.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --workload config5 --steps 200 --warmup 20 --latency-iters 300 --cpu-seconds 5 > gpurun_out/r01v.c5.log 2>&1; rc=$?; echo c5_rc=$rc; tail -1 gpurun_out/r01v.c5.log | cut -c1-2500
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --workload config3 --steps 100 --warmup 10 --latency-iters 50 --no-cpu-baseline > gpurun_out/r01v.c3.log 2>&1; rc=$?; echo c3_rc=$rc; tail -1 gpurun_out/r01v.c3.log | cut -c1-2500
exit $rc
