#!/bin/bash
# the current tree: fused-kernel + pipeline tests (int-LUT variants removed), then issue-priority A/Bs on the
# driver's command: ensemble_prio 1 vs default, feature_prio 1 vs default
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s15}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ensemble.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -40 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
FD_BENCH_SECONDARY=0 bash tools/gpu/ab5.sh $T.e "" "--engine-option ensemble_prio=1" || exit 1
FD_BENCH_SECONDARY=0 bash tools/gpu/ab5.sh $T.f "" "--engine-option feature_prio=1" || exit 1
