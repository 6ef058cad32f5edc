#!/bin/bash
# key-bucket bin index in the fused kernel's compact binning: parity tests, then the previous library (ab_prev)
# against the new on the driver's command and 200 steps, alternating
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s32}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_avg_us']; r=d['roofline']; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], {a[:8]: b for a, b in k.items()}, r.get('alone',{}).get('kernel_avg_us'), r['alone']['frac'], d['parity_vs_oracle']['timed_path']['max_abs_prob_diff'], d['parity_vs_oracle']['timed_path']['decision_mismatches'], d['parity_vs_oracle']['twin'].get('vector_mismatched_elements'))" "$1"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_configs.py tests/test_gpu_ensemble.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -40 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
PREV="FDENGINE_LIB=$PWD/realtime-fraud-detection_amd/lib/libfdengine_prev.so FDENGINE_SRC_ROOT=$PWD/ab_prev/realtime-fraud-detection_amd FDENGINE_SRC_REPO=$PWD/ab_prev"
X="--no-cpu-baseline --loaded-iters 0 --latency-iters 0"
export FD_BENCH_SECONDARY=0
for r in 1 2; do
  for v in P N; do
    [ $v = P ] && E="$PREV" || E=""
    env $E timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $X > gpurun_out/$T.$v$r.json 2> gpurun_out/$T.$v$r.log || { tail -5 gpurun_out/$T.$v$r.log; exit 1; }
    echo "[$v 20]"; summ gpurun_out/$T.$v$r.json
  done
done
for v in P N; do
  [ $v = P ] && E="$PREV" || E=""
  env $E timeout -k 10 300 python3 -u bench.py --steps 200 $X > gpurun_out/$T.${v}200.json 2> gpurun_out/$T.${v}200.log || { tail -5 gpurun_out/$T.${v}200.log; exit 1; }
  echo "[$v 200]"; summ gpurun_out/$T.${v}200.json
done
