#!/bin/bash
# PMC passes over a short bench run, one rocprofv3 --pmc call per pass (counters are never split over passes;
# each pass stays within the per-block slot limits: <= 8 SQ, <= 4 TCC, <= 2 GRBM).
#   tools/pmc.sh TAG [bench args...]      -> gpurun_out/TAG.pmc<k>/ + gpurun_out/TAG.pmc_summary.txt
# Build HERE first (the box never compiles). Each pass has its own hard time limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${1:-pmc}
shift
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--workload config3 --steps 10 --warmup 3 --no-cpu-baseline --latency-iters 2)

PASSES=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
k=0
for p in "${PASSES[@]}"; do
  k=$((k + 1))
  echo "=== pass $k: $p ($(date +%T))"
  timeout -s KILL 240 rocprofv3 --pmc $p --output-format csv -d "$OUT/$TAG.pmc$k" -o run -- \
      python "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/$TAG.pmc$k.log" 2>&1
  rc=$?
  echo "=== pass $k rc=$rc"
  tail -n 3 "$OUT/$TAG.pmc$k.log"
  [ $rc -ne 0 ] && exit $rc
done
python "$ROOT/tools/pmc_summary.py" "$OUT/$TAG".pmc* > "$OUT/$TAG.pmc_summary.txt" 2>&1
cat "$OUT/$TAG.pmc_summary.txt"
