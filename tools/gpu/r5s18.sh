#!/bin/bash
# slot_prio 1 vs 0 (the slot kernel's waves at issue priority 2): 3 x 200 steps alternating + 2 x the driver's command
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s18}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_avg_us']; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], {a[:8]: b for a, b in k.items()}, d['parity_vs_oracle']['timed_path']['max_abs_prob_diff'])" "$1"; }
X="--no-cpu-baseline --loaded-iters 0 --latency-iters 0"
for r in 1 2 3; do
  for v in O N; do
    [ $v = N ] && o="--engine-option slot_prio=1" || o=""
    FD_BENCH_SECONDARY=0 timeout -k 10 300 python3 -u bench.py --steps 200 $X $o > gpurun_out/$T.$v$r.json 2> gpurun_out/$T.$v$r.log || { tail -5 gpurun_out/$T.$v$r.log; exit 1; }
    echo "[$v 200]"; summ gpurun_out/$T.$v$r.json
  done
done
for r in 1 2; do
  for v in O N; do
    [ $v = N ] && o="--engine-option slot_prio=1" || o=""
    FD_BENCH_SECONDARY=0 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $X $o > gpurun_out/$T.d$v$r.json 2> gpurun_out/$T.d$v$r.log || { tail -5 gpurun_out/$T.d$v$r.log; exit 1; }
    echo "[$v 20]"; summ gpurun_out/$T.d$v$r.json
  done
done
