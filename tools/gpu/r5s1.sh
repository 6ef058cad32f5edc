#!/bin/bash
# ensemble_flow: GPU parity (fused kernel tests, pipelined stream), per-wave phases both schedules, driver-command A/B
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s1}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ensemble.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest_ens.log 2>&1 || { tail -40 gpurun_out/$T.pytest_ens.log; exit 1; }
tail -1 gpurun_out/$T.pytest_ens.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest_pipe.log 2>&1 || { tail -40 gpurun_out/$T.pytest_pipe.log; exit 1; }
tail -1 gpurun_out/$T.pytest_pipe.log
for o in 1 0; do
  OPTS=ensemble_flow=$o CARDS=100000000 STEPS=200 timeout -k 10 400 python3 -u tools/ens_phases_pipe.py > gpurun_out/$T.ens_phases.$o.txt 2> gpurun_out/$T.ens_phases.$o.log || { tail -20 gpurun_out/$T.ens_phases.$o.log; exit 1; }
  echo "== flow $o"; cat gpurun_out/$T.ens_phases.$o.txt
done
bash tools/gpu/ab5.sh $T "--engine-option ensemble_flow=0" "--engine-option ensemble_flow=1"
