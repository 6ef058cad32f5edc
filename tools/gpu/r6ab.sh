#!/bin/bash
# lstm_kernel4's inline searches: their first loads behind the weights (tree) vs ahead of them (ab_prev): latency
# tests, then config 5 alternating the two libraries, two rounds
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6ab}
PREV="FDENGINE_LIB=$PWD/realtime-fraud-detection_amd/lib/libfdengine_prev.so FDENGINE_SRC_ROOT=$PWD/ab_prev/realtime-fraud-detection_amd FDENGINE_SRC_REPO=$PWD/ab_prev"
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d.get('kernel_avg_us'); p=(d.get('parity_vs_oracle') or {}).get('timed_path', {}); print(sys.argv[1], round(d['value']/1e6,2), d['ms_per_step'], d.get('p99_batch_latency_ms'), k, p.get('max_abs_prob_diff'), p.get('decision_mismatches'))" "$1"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_latency.py tests/test_gpu_lstm.py tests/test_gpu_configs.py -k "latency or lstm or config5 or prebin" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
X="--workload config5 --no-cpu-baseline --loaded-iters 0 --alone-iters 0 --latency-iters 50"
for r in 1 2; do
  for v in P N; do
    [ $v = P ] && E="$PREV" || E=""
    env $E timeout -k 10 300 python3 -u bench.py $X > gpurun_out/$T.$v$r.json 2> gpurun_out/$T.$v$r.log || { tail -5 gpurun_out/$T.$v$r.log; exit 1; }
    echo "[$v$r]"; summ gpurun_out/$T.$v$r.json
  done
done
