cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
VARIANT=3 timeout -k 10 300 python tools/forest_phases.py > gpurun_out/r01t.phases.log 2>&1; rc=$?; echo phases_rc=$rc; tail -9 gpurun_out/r01t.phases.log
[ $rc -ne 0 ] && exit $rc
VARS=3 bash tools/pmc_lds.sh r01t > gpurun_out/r01t.pmc.log 2>&1; rc=$?; echo pmc_rc=$rc; cat gpurun_out/r01t.pmc.log
exit $rc
