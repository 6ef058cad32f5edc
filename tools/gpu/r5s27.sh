#!/bin/bash
# lstm_kernel4 A/B (previous library in ab_prev against the new): LSTM / latency / pipeline tests on the new one,
# W_hh 0 skipped): LSTM / latency / pipeline tests, then config 5 alternating the previous library (ab_prev) and the new
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s27}
export FD_BENCH_SECONDARY=0
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lstm.py \
    tests/test_gpu_latency.py "tests/test_gpu_pipeline.py::test_pipelined_lstm_and_latency_batches" \
    > gpurun_out/$T.pytest.txt 2>&1 || { tail -30 gpurun_out/$T.pytest.txt; exit 1; }
tail -2 gpurun_out/$T.pytest.txt
PREV="FDENGINE_LIB=$PWD/realtime-fraud-detection_amd/lib/libfdengine_prev.so FDENGINE_SRC_ROOT=$PWD/ab_prev/realtime-fraud-detection_amd FDENGINE_SRC_REPO=$PWD/ab_prev"
for r in 1 2; do
  for v in P N; do
    [ $v = P ] && E="$PREV" || E=""
    env $E timeout -k 10 300 python3 -u bench.py --workload config5 --steps 200 --no-cpu-baseline > gpurun_out/$T.$v$r.json 2> gpurun_out/$T.$v$r.log || { tail -5 gpurun_out/$T.$v$r.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], round(d['value']/1e6,2), d['ms_per_step'], d['p99_batch_latency_ms'], d['kernel_avg_us'], r['kernel_avg_us'], r['frac'], r['alone']['kernel_avg_us'], d['parity_vs_oracle']['timed_path']['max_abs_prob_diff'], d['parity_vs_oracle']['timed_path']['decision_mismatches'])" gpurun_out/$T.$v$r.json
  done
done
