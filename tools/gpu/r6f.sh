#!/bin/bash
# host cost per HIP call (microbenchmark), then the fused kernel's per-wave phases in the pipeline and alone
# (profiling build), config-4 shapes at 100 M cards
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6f}
timeout -k 10 120 ./tools/micro/hostcost > gpurun_out/$T.hostcost.txt 2>&1 || { cat gpurun_out/$T.hostcost.txt; exit 1; }
cat gpurun_out/$T.hostcost.txt
CARDS=100000000 STEPS=200 timeout -k 10 500 python3 -u tools/ens_phases_pipe.py > gpurun_out/$T.ens_phases.txt 2> gpurun_out/$T.ens_phases.log || { tail -20 gpurun_out/$T.ens_phases.log; exit 1; }
cat gpurun_out/$T.ens_phases.txt
