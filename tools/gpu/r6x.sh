#!/bin/bash
# config 5: latency_prebin 2 (binning workgroups after the LSTM's) vs 3 (searches inside the LSTM's workgroups); latency tests first
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6r}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d.get('kernel_avg_us'); print(sys.argv[1], round(d['value']/1e6,2), d['ms_per_step'], d.get('p50_batch_latency_ms'), d.get('p99_batch_latency_ms'), k, (d.get('parity_vs_oracle') or {}).get('timed_path', {}).get('max_abs_prob_diff'))" "$1"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_latency.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
X="--workload config5 --no-cpu-baseline --loaded-iters 0 --alone-iters 0 --latency-iters 50"
for r in 1 2; do
  for v in 2 3; do
    timeout -k 10 300 python3 -u bench.py $X --engine-option latency_prebin=$v > gpurun_out/$T.p$v.$r.json 2> gpurun_out/$T.p$v.$r.log || { tail -5 gpurun_out/$T.p$v.$r.log; exit 1; }
    echo "[latency_prebin=$v]"; summ gpurun_out/$T.p$v.$r.json
  done
done
