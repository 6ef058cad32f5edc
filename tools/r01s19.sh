#!/bin/bash
# per-feature binning steps: forest parity tests, XGB/IF sweeps, config 2/3/5 bench lines (no CPU leg)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s19}
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > gpurun_out/$T.$name.log 2>&1; local rc=$?
  echo "$name rc=$rc $(date +%T)"; tail -4 gpurun_out/$T.$name.log | cut -c1-300
  return $rc
}
step pytest 600 python -u -m pytest tests/test_gpu_forest.py tests/test_gpu_dropin.py tests/test_gpu_lstm.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
VARIANTS=8,3 step sweep 300 python tools/forest_sweep.py || exit 1
for wl in config2 config3 config5; do
  step bench_$wl 300 python bench.py --workload $wl --no-cpu-baseline || exit 1
done
echo done
