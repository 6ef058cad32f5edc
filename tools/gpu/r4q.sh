#!/bin/bash
# round 4: HIP API host cost of the native sharded step (rocprofv3 --hip-trace --stats over route_overhead native)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4q}
VARIANTS=native STEPS=200 CARDS=4000000 timeout -k 10 400 rocprofv3 --hip-trace --stats --output-format csv -d /tmp/$T.prof -o run -- \
  python tools/route_overhead.py > gpurun_out/$T.log 2>&1 || exit $?
for f in $(find /tmp/$T.prof -name "*stats.csv" -o -name "*hip_api_trace.csv"); do cp "$f" gpurun_out/$T.$(basename $f); done
ls gpurun_out | grep $T
rm -rf /tmp/$T.prof
