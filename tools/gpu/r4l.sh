#!/bin/bash
# round 4: every workload's bench line, then PMC of config 4 / 5 and the ingest kernel
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4l}
WORKLOADS="config2 config3 config5 ingest config3j" bash tools/gpu/workloads.sh $T || exit 1
bash tools/gpu/pmc_r04.sh $T || exit 1
bash tools/gpu/pmc_ingest.sh $T || exit 1
