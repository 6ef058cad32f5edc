#!/bin/bash
# smoke -> full -m gpu suite -> default bench -> rocprof stats of the bench (raw trace reduced on the box)
# -> (PHASES=1) the ensemble kernel's phase split beside the features vs alone (profiling build)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-full}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T.smoke.log 2>&1 || exit $?
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/$T.pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$T.pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -u bench.py > gpurun_out/$T.bench.log 2>&1 || exit $?
grep '^{' gpurun_out/$T.bench.log > gpurun_out/$T.bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$T.prof -o run -- \
  python bench.py --no-cpu-baseline > gpurun_out/$T.prof.log 2>&1 || exit $?
f=$(find /tmp/$T.prof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/$T.kernel_stats.csv
rm -rf /tmp/$T.prof
if [ "${PHASES:-0}" = 1 ]; then
  timeout -k 10 300 python -u tools/ens_phases_pipe.py > gpurun_out/$T.ens_phases_pipe.log 2>&1 || exit $?
fi
if [ "${ROUTE:-0}" = 1 ]; then
  timeout -k 10 400 python -u tools/route_overhead.py > gpurun_out/$T.route_overhead.log 2>&1 || exit $?
fi
