#!/bin/bash
# the sharded step's forward worker + ensemble chunk sizes: parity (ensemble, sharding), the direct / native steps
# (worker on / off), the default bench line
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-t}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ensemble.py tests/test_gpu_sharding.py -m gpu -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -2 gpurun_out/$T.pytest.log
VARIANTS=direct,native,native_nothread timeout -k 10 300 python -u tools/route_overhead.py > gpurun_out/$T.route.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 300 --warmup 20 > gpurun_out/$T.bench.json 2> gpurun_out/$T.bench.err || exit $?
