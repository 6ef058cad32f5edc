#!/bin/bash
# sharded step with the owner's results written in place (no staging copy, one event record less): the sharded and
# routed parity tests, then the world-1 host cost against the direct step
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6g}
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharding_loopback.py tests/test_gpu_sharding.py tests/test_gpu_sharding_mp.py tests/test_gpu_pipeline.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -40 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
VARIANTS=direct,native STEPS=200 timeout -k 10 500 python3 -u tools/route_overhead.py > gpurun_out/$T.route.txt 2> gpurun_out/$T.route.log || { tail -20 gpurun_out/$T.route.log; exit 1; }
cat gpurun_out/$T.route.txt
