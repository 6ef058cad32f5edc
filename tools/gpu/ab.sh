#!/bin/bash
# A/B bench lines + pipeline tests: ab.sh TAG "pytest selection" "bench args A" "bench args B" ...
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; SEL=$2; shift 2
if [ -n "$SEL" ]; then
  timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/$T.pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$T.pytest.log; [ $rc -ne 0 ] && exit $rc
fi
k=0
for args in "$@"; do
  k=$((k + 1))
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $args > gpurun_out/$T.b$k.log 2>&1 || exit $?
  grep '^{' gpurun_out/$T.b$k.log > gpurun_out/$T.b$k.json
done
