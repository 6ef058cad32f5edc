#!/bin/bash
# IsolationForest kernel sweep + config-3 bench under a chosen forest_kernel default
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s14}
IF=1 VARIANTS=${VARIANTS:-3,8} timeout -k 10 300 python tools/forest_sweep.py > gpurun_out/$T.sweep_if.log 2>&1; rc=$?; echo sweep_if_rc=$rc; tail -3 gpurun_out/$T.sweep_if.log
[ $rc -ne 0 ] && exit $rc
VARIANTS=${VARIANTS:-3,8} timeout -k 10 300 python tools/forest_sweep.py > gpurun_out/$T.sweep.log 2>&1; rc=$?; echo sweep_rc=$rc; tail -3 gpurun_out/$T.sweep.log
exit $rc
