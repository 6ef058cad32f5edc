#!/bin/bash
# A/B of engine options on the driver's command (and 200 steps), alternating, one call. usage: ab5.sh TAG "opts A" "opts B"
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; A=$2; Bo=$3
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_avg_us']; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], {a[:8]: b for a, b in k.items()}, d.get('diag_blocks_ms_per_step'), d['parity_vs_oracle']['timed_path']['max_abs_prob_diff'], d['parity_vs_oracle']['timed_path']['decision_mismatches'])" "$1"; }
X="--no-cpu-baseline --loaded-iters 0 --alone-iters 0 --latency-iters 0"
for r in 1 2; do
  for v in A B; do
    [ $v = A ] && o="$A" || o="$Bo"
    FD_BENCH_BLOCKS=4 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $X $o > gpurun_out/$T.$v$r.json 2> gpurun_out/$T.$v$r.log || { tail -5 gpurun_out/$T.$v$r.log; exit 1; }
    echo "[$v: $o]"; summ gpurun_out/$T.$v$r.json
  done
done
for v in A B; do
  [ $v = A ] && o="$A" || o="$Bo"
  timeout -k 10 300 python3 -u bench.py --steps 200 $X $o > gpurun_out/$T.${v}200.json 2> gpurun_out/$T.${v}200.log || { tail -5 gpurun_out/$T.${v}200.log; exit 1; }
  echo "[$v 200: $o]"; summ gpurun_out/$T.${v}200.json
done
