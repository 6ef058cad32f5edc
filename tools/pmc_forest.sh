#!/bin/bash
# PMC passes (one counter group per pass, --kernel-trace only) for the forest kernel on config 2.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-pmc}
timeout -k 10 120 rocprofv3 -L > gpurun_out/$TAG.counters.txt 2>&1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/$TAG.p$i -o run -- \
     python tools/forest_sweep.py > gpurun_out/$TAG.p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
exit 0
