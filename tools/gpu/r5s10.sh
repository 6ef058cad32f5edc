#!/bin/bash
# count exchange as one all-gather (default) vs 2 x world sends / receives: sharding GPU tests (loopback world 2/4/8,
# real RCCL world 1), the world-1 native step A/B (route_overhead, alternating), loopback host phases per world
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s10}
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharding_loopback.py tests/test_gpu_sharding.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -40 gpurun_out/$T.pytest.log; exit 1; }
grep -c PASSED gpurun_out/$T.pytest.log; tail -1 gpurun_out/$T.pytest.log
for r in 1 2; do
  for ce in 0 1; do
    COUNT_EXCHANGE=$ce VARIANTS=direct,native STEPS=200 timeout -k 10 300 python3 -u tools/route_overhead.py > gpurun_out/$T.ro.$ce.$r.log 2>&1 || { tail -20 gpurun_out/$T.ro.$ce.$r.log; exit 1; }
    echo "[count_exchange $ce run $r]"; grep -E "ms/step|host us|/ direct" gpurun_out/$T.ro.$ce.$r.log
  done
done
for ce in 0 1; do
  COUNT_EXCHANGE=$ce timeout -k 10 400 python3 -u tools/loopback_host.py 1,2,4,8 16384 40 > gpurun_out/$T.lh.$ce.log 2>&1 || { tail -20 gpurun_out/$T.lh.$ce.log; exit 1; }
  echo "[loopback host, count_exchange $ce]"; grep '^{"world' gpurun_out/$T.lh.$ce.log | cut -c1-400
done
