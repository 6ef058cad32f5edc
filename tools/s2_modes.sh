# pipeline parity tests, then bench A/B over pipeline modes (+ rocprof trace of mode 2)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-s2m}
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1; rc=$?; tail -4 gpurun_out/$T.pytest.log; [ $rc -ne 0 ] && exit $rc
for m in 1 2; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --latency-iters 50 --pipeline-mode $m > gpurun_out/$T.mode$m.log 2>&1 || exit $?
  grep '^{' gpurun_out/$T.mode$m.log > gpurun_out/$T.mode$m.json
  python3 -c "import json; d=json.load(open('gpurun_out/$T.mode$m.json')); print('mode $m', round(d['value']/1e6,2), d['ms_per_step'], d.get('host_submit_ms_per_step'), d['p99_batch_latency_ms'], d['kernel_avg_us'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T.prof2 -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 10 --pipeline-mode 2 > gpurun_out/$T.rocprof2.log 2>&1 || exit $?
echo done
