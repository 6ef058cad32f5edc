#!/bin/bash
# round 4: the native sharded step vs the direct one after the VGPR fix (host phases), ingest phases
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4p}
VARIANTS=direct,native timeout -k 10 400 python -u tools/route_overhead.py > gpurun_out/$T.route_overhead.log 2>&1 || exit $?
grep -E "ms/step|host us|direct" gpurun_out/$T.route_overhead.log
timeout -k 10 300 python -u tools/ingest_phases.py > gpurun_out/$T.ingest_phases.log 2>&1 || exit 1
grep stop_after gpurun_out/$T.ingest_phases.log
