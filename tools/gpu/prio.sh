#!/bin/bash
# stream priorities (engine option stream_priority) vs the direct and native steps
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-p}
for P in ${PRIOS:-0 1 2 3}; do
  echo "== stream_priority=$P" >> gpurun_out/$T.prio.log
  STREAM_PRIORITY=$P VARIANTS=${VARIANTS:-direct,native,native_nothread} timeout -k 10 300 python -u tools/route_overhead.py >> gpurun_out/$T.prio.log 2>&1 || exit $?
done
