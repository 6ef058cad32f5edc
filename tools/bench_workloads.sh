# bench lines for non-default workloads (WORKLOADS), pipelined and --no-pipeline (VARIANTS), after the GPU tests in TESTS
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-wl}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_pipeline.py} -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1; rc=$?; tail -4 gpurun_out/$T.pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for wl in ${WORKLOADS:-config3 config5 config3j}; do
  for v in ${VARIANTS:-pipe serial}; do
    extra=""; [ $v = serial ] && extra="--no-pipeline"
    timeout -k 10 400 python bench.py --workload $wl --steps 200 --warmup 20 $extra ${BENCH_ARGS:-} > gpurun_out/$T.$wl.$v.log 2>&1 || exit $?
    grep '^{' gpurun_out/$T.$wl.$v.log > gpurun_out/$T.$wl.$v.json
    V="$wl $v" python3 -c "import json,os; d=json.load(open('gpurun_out/$T.$wl.$v.json')); print(os.environ['V'], round(d['value']/1e6,2), d['ms_per_step'], d.get('host_submit_ms_per_step'), d['p99_batch_latency_ms'], d['kernel_avg_us'], d['roofline'].get('frac'), d['parity_vs_oracle'])"
  done
done
echo done
