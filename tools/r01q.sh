cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
WL=config2 bash tools/pmc_bench.sh r01q > gpurun_out/r01q.pmc2.log 2>&1; rc=$?; echo pmc2_rc=$rc; tail -30 gpurun_out/r01q.pmc2.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --workload config3 --steps 100 --warmup 10 --latency-iters 50 --cpu-seconds 8 > gpurun_out/r01q.c3.log 2>&1; rc=$?; echo c3_rc=$rc; tail -3 gpurun_out/r01q.c3.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01q.c3prof -o run -- python bench.py --workload config3 --steps 50 --warmup 5 --latency-iters 5 --no-cpu-baseline > gpurun_out/r01q.c3prof.log 2>&1; rc=$?; echo c3prof_rc=$rc
exit $rc
