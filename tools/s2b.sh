# round-2 session-2 pipeline check: parity tests, then bench A/B (pipelined / serial), rocprof stats
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-s2b}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_pipeline.py} -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1; rc=$?; tail -8 gpurun_out/$T.pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for v in ${VARIANTS:-pipe serial}; do
  extra=""; [ $v = serial ] && extra="--no-pipeline"
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --latency-iters 50 $extra ${BENCH_ARGS:-} > gpurun_out/$T.bench_$v.log 2>&1 || exit $?
  grep '^{' gpurun_out/$T.bench_$v.log | V=$v python3 -c "import json,sys,os; d=json.loads(sys.stdin.read()); print(os.environ['V'], d['value']/1e6, d['ms_per_step'], d['host_submit_ms_per_step'], d['p99_batch_latency_ms'], d['kernel_avg_us'], d['parity_vs_oracle'])"
done
if [ "${PROFILE:-1}" = 1 ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T.prof -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 10 ${BENCH_ARGS:-} > gpurun_out/$T.rocprof.log 2>&1 || exit $?
fi
echo done
