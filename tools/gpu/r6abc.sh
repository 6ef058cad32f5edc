#!/bin/bash
# three libraries alternating on the driver's command and 200 steps: P (ab_prev), A (ab_A), N (the tree's)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-abc}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_avg_us']; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], {a[:8]: b for a, b in k.items()}, (d.get('parity_vs_oracle') or {}).get('timed_path', {}).get('max_abs_prob_diff'))" "$1"; }
L=$PWD/realtime-fraud-detection_amd/lib
EP="FDENGINE_LIB=$L/libfdengine_prev.so FDENGINE_SRC_ROOT=$PWD/ab_prev/realtime-fraud-detection_amd FDENGINE_SRC_REPO=$PWD/ab_prev"
EA="FDENGINE_LIB=$L/libfdengine_A.so FDENGINE_SRC_ROOT=$PWD/ab_A/realtime-fraud-detection_amd FDENGINE_SRC_REPO=$PWD/ab_A"
X="--no-cpu-baseline --loaded-iters 0 --latency-iters 0 --alone-iters 0"
export FD_BENCH_SECONDARY=0
for r in 1 2; do
  for v in P A N; do
    [ $v = P ] && E="$EP"; [ $v = A ] && E="$EA"; [ $v = N ] && E=""
    env $E timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $X > gpurun_out/$T.$v$r.json 2> gpurun_out/$T.$v$r.log || { tail -5 gpurun_out/$T.$v$r.log; exit 1; }
    echo "[$v 20]"; summ gpurun_out/$T.$v$r.json
  done
done
for v in P A N; do
  [ $v = P ] && E="$EP"; [ $v = A ] && E="$EA"; [ $v = N ] && E=""
  env $E timeout -k 10 300 python3 -u bench.py --steps 200 $X > gpurun_out/$T.${v}200.json 2> gpurun_out/$T.${v}200.log || { tail -5 gpurun_out/$T.${v}200.log; exit 1; }
  echo "[$v 200]"; summ gpurun_out/$T.${v}200.json
done
