#!/bin/bash
# Round-1 closing check: smoke, full GPU parity suite, default bench line; PMC passes: HBM traffic /
# L2 hit rate for every config-3 kernel (features, forests, blend) and MFMA busy cycles for config 5.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s18}
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > gpurun_out/$T.$name.log 2>&1; local rc=$?
  echo "$name rc=$rc $(date +%T)"; tail -1 gpurun_out/$T.$name.log | cut -c1-200
  return $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
step bench 400 python bench.py || exit 1
WL=config3 step pmc3 600 bash tools/pmc_bench.sh $T.pmc || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
  -d gpurun_out/$T.mfma5 -o run -- python bench.py --workload config5 --steps 20 --warmup 3 --latency-iters 0 --no-cpu-baseline \
  > gpurun_out/$T.mfma5.log 2>&1; echo "mfma5 rc=$?"
echo done
