#!/bin/bash
# world-1 sharded host cost, previous library (ab_prev: staged results + copy kernel) against the tree's, alternating
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6h}
PREV="FDENGINE_LIB=$PWD/realtime-fraud-detection_amd/lib/libfdengine_prev.so FDENGINE_SRC_ROOT=$PWD/ab_prev/realtime-fraud-detection_amd FDENGINE_SRC_REPO=$PWD/ab_prev"
timeout -k 10 120 ./tools/micro/hostcost > gpurun_out/$T.hostcost.txt 2>&1 || { cat gpurun_out/$T.hostcost.txt; exit 1; }
cat gpurun_out/$T.hostcost.txt
for r in 1 2; do
  for v in P N; do
    [ $v = P ] && E="$PREV" || E=""
    env $E VARIANTS=direct,native STEPS=200 timeout -k 10 500 python3 -u tools/route_overhead.py > gpurun_out/$T.$v$r.txt 2> gpurun_out/$T.$v$r.log || { tail -20 gpurun_out/$T.$v$r.log; exit 1; }
    echo "== $v$r"; grep -v "^Hostname\|^Librccl" gpurun_out/$T.$v$r.txt
  done
done
