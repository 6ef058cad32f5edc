#!/bin/bash
# latency_prebin 3 as the default: latency / pipeline / config tests, then config 5 twice (default) and once at 2
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6y}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d.get('kernel_avg_us'); p=(d.get('parity_vs_oracle') or {}).get('timed_path', {}); print(sys.argv[1], round(d['value']/1e6,2), d['ms_per_step'], d.get('p99_batch_latency_ms'), k, p.get('max_abs_prob_diff'), p.get('decision_mismatches'))" "$1"; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_latency.py tests/test_gpu_pipeline.py tests/test_gpu_configs.py tests/test_gpu_lstm.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
X="--workload config5 --no-cpu-baseline --loaded-iters 0 --alone-iters 0 --latency-iters 100"
for v in d 2 d; do
  O=""; [ $v = 2 ] && O="--engine-option latency_prebin=2"
  timeout -k 10 300 python3 -u bench.py $X $O > gpurun_out/$T.$v.json 2> gpurun_out/$T.$v.log || { tail -5 gpurun_out/$T.$v.log; exit 1; }
  echo "[$v]"; summ gpurun_out/$T.$v.json
done
