cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python bench.py --workload ingest --steps 200 --warmup 10 --cpu-seconds 8 > gpurun_out/s3.ingest.log 2>&1; rc=$?; echo ingest_rc=$rc; tail -2 gpurun_out/s3.ingest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s3.ingprof -o run -- python bench.py --workload ingest --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 10 > gpurun_out/s3.ingprof.log 2>&1; rc=$?; echo ingprof_rc=$rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py --workload config3j --steps 100 --warmup 10 --cpu-seconds 8 --latency-iters 100 > gpurun_out/s3.c3j.log 2>&1; rc=$?; echo c3j_rc=$rc; tail -2 gpurun_out/s3.c3j.log
exit $rc
