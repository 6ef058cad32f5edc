#!/bin/bash
# A/B of the native sharded step's host cost in ONE call (host speed differs between boxes): lib/variants/*_A.so
# (FDENGINE_LIB, build-id check off) against the tree's library, alternating A B A B
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-abn}
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then
      FDENGINE_LIB=$PWD/realtime-fraud-detection_amd/lib/variants/libfdengine_A.so FDENGINE_SRC_ROOT=/nonexistent \
        VARIANTS=direct,native STEPS=300 timeout -k 10 400 python -u tools/route_overhead.py > gpurun_out/$T.$v$r.log 2>&1 || exit $?
    else
      VARIANTS=direct,native STEPS=300 timeout -k 10 400 python -u tools/route_overhead.py > gpurun_out/$T.$v$r.log 2>&1 || exit $?
    fi
    echo "== $v$r"; grep -E "ms/step|host us" gpurun_out/$T.$v$r.log
  done
done
