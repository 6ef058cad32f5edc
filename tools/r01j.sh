cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python bench.py --workload config3 --steps 100 --warmup 10 --latency-iters 50 > gpurun_out/r01j.bench3.log 2>&1; rc=$?; echo bench3_rc=$rc; tail -3 gpurun_out/r01j.bench3.log
[ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01j.prof3 -o run -- python bench.py --workload config3 --steps 50 --warmup 5 --latency-iters 5 --no-cpu-baseline > gpurun_out/r01j.rocprof3.log 2>&1; echo rocprof_rc=$?
