#!/bin/bash
# ensemble_stage_hi: fused-kernel + pipeline tests, per-wave phases 0 / 1, driver's command A/B
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s14}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ensemble.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -40 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
for o in 1 0; do
  OPTS=ensemble_stage_hi=$o CARDS=100000000 STEPS=100 timeout -k 10 400 python3 -u tools/ens_phases_pipe.py > gpurun_out/$T.ens_phases.$o.txt 2> gpurun_out/$T.ens_phases.$o.log || { tail -20 gpurun_out/$T.ens_phases.$o.log; exit 1; }
  echo "== stage_hi $o"; grep -E "^beside|^alone|prologue  |total|marks|span" gpurun_out/$T.ens_phases.$o.txt
done
FD_BENCH_SECONDARY=0 bash tools/gpu/ab5.sh $T "--engine-option ensemble_stage_hi=0" "--engine-option ensemble_stage_hi=1"
