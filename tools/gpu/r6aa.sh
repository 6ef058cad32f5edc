#!/bin/bash
# the split-row ring released by the scoring-done events (a ring of four) instead of an event of its own on the
# engine stream: twin / loopback / config tests, then the previous library (ab_prev) against the tree's, alternating:
# the driver's command, 200 steps, and the world-1 sharded step's host cost
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6aa}
PREV="FDENGINE_LIB=$PWD/realtime-fraud-detection_amd/lib/libfdengine_prev.so FDENGINE_SRC_ROOT=$PWD/ab_prev/realtime-fraud-detection_amd FDENGINE_SRC_REPO=$PWD/ab_prev"
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_avg_us']; h=d.get('host_submit_breakdown') or {}; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], d.get('host_submit_ms_per_step'), h.get('native_us_per_step'), {a[:8]: b for a, b in k.items()}, (d.get('parity_vs_oracle') or {}).get('timed_path', {}).get('max_abs_prob_diff'))" "$1"; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_sharding_loopback.py tests/test_gpu_configs.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
X="--no-cpu-baseline --loaded-iters 0 --latency-iters 0 --alone-iters 0"
export FD_BENCH_SECONDARY=0
for r in 1 2; do
  for v in P N; do
    [ $v = P ] && E="$PREV" || E=""
    env $E timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $X > gpurun_out/$T.$v$r.json 2> gpurun_out/$T.$v$r.log || { tail -5 gpurun_out/$T.$v$r.log; exit 1; }
    echo "[20 $v]"; summ gpurun_out/$T.$v$r.json
  done
done
for v in P N; do
  [ $v = P ] && E="$PREV" || E=""
  env $E timeout -k 10 300 python3 -u bench.py --steps 200 $X > gpurun_out/$T.${v}200.json 2> gpurun_out/$T.${v}200.log || { tail -5 gpurun_out/$T.${v}200.log; exit 1; }
  echo "[200 $v]"; summ gpurun_out/$T.${v}200.json
done
for v in P N; do
  [ $v = P ] && E="$PREV" || E=""
  env $E VARIANTS=direct,native STEPS=200 timeout -k 10 400 python3 -u tools/route_overhead.py > gpurun_out/$T.ro$v.txt 2> gpurun_out/$T.ro$v.log || { tail -20 gpurun_out/$T.ro$v.log; exit 1; }
  echo "== route_overhead $v"; grep -v "^Hostname\|^Librccl\|version" gpurun_out/$T.ro$v.txt
done
