#!/bin/bash
# round 4: records + next counts in one RCCL group: sharded-step tests (loopback world 2/4, world 1 RCCL), host cost
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4r}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sharding_loopback.py tests/test_gpu_sharding.py tests/test_gpu_sharding_mp.py \
  > gpurun_out/$T.pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$T.pytest.log; [ $rc -ne 0 ] && exit $rc
VARIANTS=direct,native timeout -k 10 400 python -u tools/route_overhead.py > gpurun_out/$T.route_overhead.log 2>&1 || exit $?
grep -E "ms/step|host us|direct" gpurun_out/$T.route_overhead.log
