#!/bin/bash
# One gpurun call: build check, smoke, GPU parity tests, bench, rocprofv3 kernel trace.
# Each GPU step has its own time limit; a crash / fault / timeout ends the script (no retries).
# Test FAILURES (pytest exit 1) do not stop the bench; anything else non-zero does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TAG=${1:-run}
STEPS=${STEPS:-200}

run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$TAG.$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "$OUT/$TAG.$name.log"
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ] && [ "$1" -ne 5 ]; }

run build 900 python -c "import __graft_entry__ as g; g.build()"; rc=$?; fatal $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
run smoke 600 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; fatal $rc && exit $rc
run pytest_gpu 1200 python -m pytest tests -m gpu -x -q -p no:cacheprovider; rc=$?; fatal $rc && exit $rc
run bench 900 python bench.py --steps "$STEPS" --warmup 20; rc=$?; fatal $rc && exit $rc
grep '^{' "$OUT/$TAG.bench.log" > "$OUT/$TAG.bench.json" || true
if [ "${PROFILE:-1}" = "1" ]; then
  export TMPDIR=/tmp
  run rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$TAG.prof" -o run -- \
      python "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 10; rc=$?
  fatal $rc && exit $rc
fi
echo "=== done"
