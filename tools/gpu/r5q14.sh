#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q14}
CARDS=100000000 STEPS=200 timeout -k 10 400 python3 -u tools/ens_phases_pipe.py > gpurun_out/$T.ens_phases.txt 2> gpurun_out/$T.ens_phases.log || { tail -20 gpurun_out/$T.ens_phases.log; exit 1; }
cat gpurun_out/$T.ens_phases.txt
