#!/bin/bash
# One gpurun call (build HERE first: the box runs the in-tree .so, it never compiles):
#   tools/gpu_check.sh TAG            smoke -> pytest -m gpu -> bench (default workload) -> rocprofv3 --stats
# Environment knobs: STEPS (bench steps, 200), TESTS (pytest selection, "tests"), SKIP_TESTS=1,
#   WORKLOADS="config2 config3 ..." (extra bench lines), PROFILE=0 (no rocprof pass), PYTEST_K (-k expr).
# Each GPU step has its own time limit; a crash / fault / timeout ends the script (no retries).
# Test FAILURES (pytest exit 1) do not stop the bench; anything else non-zero does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${1:-run}
STEPS=${STEPS:-200}

run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$TAG.$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 4 "$OUT/$TAG.$name.log"
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ] && [ "$1" -ne 5 ]; }

run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; fatal $rc && exit $rc
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  run pytest_gpu 1100 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread \
      -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"}; rc=$?; fatal $rc && exit $rc
fi
run bench 900 python bench.py --steps "$STEPS" --warmup 20; rc=$?; fatal $rc && exit $rc
grep '^{' "$OUT/$TAG.bench.log" > "$OUT/$TAG.bench.json" || true
for wl in ${WORKLOADS:-}; do
  run "bench_$wl" 600 python bench.py --workload "$wl" --steps "$STEPS" --warmup 20; rc=$?; fatal $rc && exit $rc
  grep '^{' "$OUT/$TAG.bench_$wl.log" > "$OUT/$TAG.$wl.bench.json" || true
done
if [ "${PROFILE:-1}" = "1" ]; then
  FD_BENCH_SECONDARY=0 run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$TAG.prof" -o run -- \
      python "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 10; rc=$?
  fatal $rc && exit $rc
fi
echo "=== done"
