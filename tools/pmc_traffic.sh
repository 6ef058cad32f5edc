# HBM traffic (FETCH_SIZE / WRITE_SIZE passes, one rocprofv3 --pmc run each) of the default bench + config5 line
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-pmc}
k=0
for p in FETCH_SIZE WRITE_SIZE; do
  k=$((k + 1))
  timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d gpurun_out/$T.pmc$k -o run -- \
      python bench.py --steps 10 --warmup 3 --no-cpu-baseline --latency-iters 2 --parity-batches 1 > gpurun_out/$T.pmc$k.log 2>&1 || exit $?
  echo "pass $k ok"
done
python3 tools/pmc_json.py config4 65536 ensemble_kernel gpurun_out/$T.pmc_config4.json gpurun_out/$T.pmc1 gpurun_out/$T.pmc2 || exit $?
head -8 gpurun_out/$T.pmc_config4.json
timeout -k 10 400 python bench.py --workload config5 --steps 200 --warmup 20 > gpurun_out/$T.config5.log 2>&1 || exit $?
grep '^{' gpurun_out/$T.config5.log > gpurun_out/$T.config5.json
python3 -c "import json; d=json.load(open('gpurun_out/$T.config5.json')); print('config5', round(d['value']/1e6,2), d['ms_per_step'], d.get('host_submit_ms_per_step'), d['p99_batch_latency_ms'], d['kernel_avg_us'])"
echo done
