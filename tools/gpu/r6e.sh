#!/bin/bash
# A/B of the previous library (ab_prev) against the tree's: parity tests of the fused kernel, then the driver's
# command x2 alternating, 200 steps, and config 2 (the fused single-forest kernel), each with the kernels alone
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6e}; TESTS=${TESTS:-tests/test_gpu_ensemble.py tests/test_gpu_pipeline.py}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_avg_us']; r=d['roofline']; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], {a[:8]: b for a, b in k.items()}, (r.get('alone') or {}).get('kernel_avg_us'), (r.get('alone') or {}).get('frac'), (d.get('parity_vs_oracle') or {}).get('timed_path', {}).get('max_abs_prob_diff'))" "$1"; }
timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -40 gpurun_out/$T.pytest.log; exit 1; }
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
  env $E timeout -k 10 300 python3 -u bench.py --workload config2 --steps 200 $X > gpurun_out/$T.${v}c2.json 2> gpurun_out/$T.${v}c2.log || { tail -5 gpurun_out/$T.${v}c2.log; exit 1; }
  echo "[$v config2]"; summ gpurun_out/$T.${v}c2.json
done
