#!/bin/bash
# LDS-pipe PMC passes for the forest kernel variants (config-2 shapes), one counter group per pass.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-lds}
for v in ${VARS:-1 2}; do
  i=0
  for grp in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
             "SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS" \
             "SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVES"; do
    i=$((i+1))
    VARIANTS=$v timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/$TAG.v$v.p$i -o run -- \
       python tools/forest_sweep.py > gpurun_out/$TAG.v$v.p$i.log 2>&1
    rc=$?; echo "v$v pass $i ($grp) rc=$rc"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
