cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
true; rc=0
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --workload config4 --steps 100 --warmup 10 --latency-iters 50 --cpu-seconds 8 > gpurun_out/r01r.c4.log 2>&1; rc=$?; echo c4_rc=$rc; tail -3 gpurun_out/r01r.c4.log
exit $rc
