#!/bin/bash
# Round-1 session-10 GPU check: smoke, full GPU parity suite, default bench line, rocprofv3 kernel stats.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s10}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T.smoke.log 2>&1; rc=$?; echo smoke_rc=$rc; tail -2 gpurun_out/$T.smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/$T.pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/$T.bench.log 2>&1; rc=$?; echo bench_rc=$rc; tail -1 gpurun_out/$T.bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T.prof -o run -- \
  python bench.py --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 10 > gpurun_out/$T.prof.log 2>&1; rc=$?; echo prof_rc=$rc; tail -1 gpurun_out/$T.prof.log
exit $rc
