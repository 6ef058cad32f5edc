#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-g}
timeout -k 10 300 python -u tools/ens_phases_pipe.py > gpurun_out/$T.ens_phases_pipe.log 2>&1 || exit $?
FD_STALL_TRACE=3 timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-iters 20 --loaded-iters 400 > gpurun_out/$T.stall.log 2>&1 || exit $?
