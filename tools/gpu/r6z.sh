#!/bin/bash
# round-6 close on the final tree: r6final.sh (smoke, every GPU test, the driver's command twice, 200 steps, rocprof)
# then the config-5 PMC summary for the current lstm_kernel4
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-fin6d}
bash tools/gpu/r6final.sh $T || exit $?
WORKLOADS=5 bash tools/gpu/pmc_r05.sh ${T}pmc || exit $?
