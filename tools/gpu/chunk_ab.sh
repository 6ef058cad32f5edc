#!/bin/bash
# ensemble chunk-size experiment: parity, the direct / native steps, the default bench line
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ensemble.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -20 gpurun_out/$T.pytest.log; exit 1; }
tail -2 gpurun_out/$T.pytest.log
VARIANTS=direct,native timeout -k 10 300 python -u tools/route_overhead.py > gpurun_out/$T.route.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 300 --warmup 20 > gpurun_out/$T.bench.json 2> gpurun_out/$T.bench.err || exit $?
