#!/bin/bash
# engine-option re-tune under split rows: each variant on the driver's command and at 200 steps, two rounds alternating
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-sw}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_avg_us']; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], {a[:8]: b for a, b in k.items()})" "$1"; }
X="--no-cpu-baseline --loaded-iters 0 --latency-iters 0 --alone-iters 0"
export FD_BENCH_SECONDARY=0
VARS=("" "--engine-option feature_prio=0" "--engine-option bucket_keys=64" "--engine-option ensemble_prio=1" "--engine-option slot_stream=0" "--engine-option slot_prio=1")
for r in 1 2; do
  for i in "${!VARS[@]}"; do
    timeout -k 10 300 python3 -u bench.py --steps 200 $X ${VARS[$i]} > gpurun_out/$T.v$i.$r.json 2> gpurun_out/$T.v$i.$r.log || { tail -5 gpurun_out/$T.v$i.$r.log; exit 1; }
    echo "[v$i ${VARS[$i]}]"; summ gpurun_out/$T.v$i.$r.json
  done
done
# config 5 (latency batches): the previous library (ab_prev) against the tree's, alternating
PREV="FDENGINE_LIB=$PWD/realtime-fraud-detection_amd/lib/libfdengine_prev.so FDENGINE_SRC_ROOT=$PWD/ab_prev/realtime-fraud-detection_amd FDENGINE_SRC_REPO=$PWD/ab_prev"
for r in 1 2; do
  for v in P N; do
    [ $v = P ] && E="$PREV" || E=""
    env $E timeout -k 10 300 python3 -u bench.py --workload config5 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/$T.c5$v$r.json 2> gpurun_out/$T.c5$v$r.log || { tail -5 gpurun_out/$T.c5$v$r.log; exit 1; }
    echo "[config5 $v$r]"; summ gpurun_out/$T.c5$v$r.json
  done
done
