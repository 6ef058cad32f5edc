#!/bin/bash
# Round-1 final measurement: smoke, full GPU parity suite, every bench workload (with the CPU leg),
# rocprofv3 kernel stats for config 2 and config 3, PMC HBM-traffic passes for config 2.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s15}
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > gpurun_out/$T.$name.log 2>&1; local rc=$?
  echo "$name rc=$rc $(date +%T)"; tail -1 gpurun_out/$T.$name.log | cut -c1-200
  return $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
for wl in config2 config3 config4 config5 ingest config3j; do
  step bench_$wl 400 python bench.py --workload $wl || exit 1
done
step prof2 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T.prof2 -o run -- \
  python bench.py --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 10 || exit 1
step prof3 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T.prof3 -o run -- \
  python bench.py --workload config3 --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 10 || exit 1
step pmc 600 bash tools/pmc_bench.sh $T.pmc || exit 1
echo done
