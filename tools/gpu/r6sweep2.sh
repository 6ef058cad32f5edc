#!/bin/bash
# issue priorities under split rows: default, feature_prio 0, ensemble_prio 1, both — driver's command (x2) and 200 steps
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-sx}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_avg_us']; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], {a[:8]: b for a, b in k.items()})" "$1"; }
X="--no-cpu-baseline --loaded-iters 0 --latency-iters 0 --alone-iters 0"
export FD_BENCH_SECONDARY=0
VARS=("" "--engine-option feature_prio=0" "--engine-option ensemble_prio=1" "--engine-option feature_prio=0 --engine-option ensemble_prio=1")
for r in 1 2; do
  for i in "${!VARS[@]}"; do
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $X ${VARS[$i]} > gpurun_out/$T.d$i.$r.json 2> gpurun_out/$T.d$i.$r.log || { tail -5 gpurun_out/$T.d$i.$r.log; exit 1; }
    echo "[20 v$i ${VARS[$i]}]"; summ gpurun_out/$T.d$i.$r.json
  done
done
for i in "${!VARS[@]}"; do
  timeout -k 10 300 python3 -u bench.py --steps 200 $X ${VARS[$i]} > gpurun_out/$T.s$i.json 2> gpurun_out/$T.s$i.log || { tail -5 gpurun_out/$T.s$i.log; exit 1; }
  echo "[200 v$i ${VARS[$i]}]"; summ gpurun_out/$T.s$i.json
done
