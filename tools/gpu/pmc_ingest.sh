#!/bin/bash
# PMC of the ingest kernel at 64 k simulator-format messages (full kernel, stop_after 0): instruction mix and
# wait cycles, one rocprofv3 --pmc pass per counter group; summary -> gpurun_out/T.pmc_ingest.json
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-pmci}
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
  "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"
)
k=0
for p in "${PASSES[@]}"; do
  k=$((k + 1))
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d /tmp/$T.p$k -o run -- \
      python tools/ingest_phases.py 0 > gpurun_out/$T.p$k.log 2>&1
  rc=$?; echo "ingest pass $k rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_kernels.py ingest 65536 ingest_json_kernel gpurun_out/$T.pmc_ingest.json /tmp/$T.p* || exit $?
rm -rf /tmp/$T.p*
