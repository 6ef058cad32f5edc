#!/bin/bash
# ensemble_bin_global: option tests, per-wave phases (both arms), A/B on the driver's command
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q19}
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 300 --timeout-method thread > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
for o in ensemble_bin_global=0 ensemble_bin_global=1; do
  OPTS=$o CARDS=100000000 STEPS=200 timeout -k 10 400 python3 -u tools/ens_phases_pipe.py > gpurun_out/$T.ens_phases.$o.txt 2> gpurun_out/$T.ens_phases.$o.log || { tail -20 gpurun_out/$T.ens_phases.$o.log; exit 1; }
  echo "== $o"; cat gpurun_out/$T.ens_phases.$o.txt
done
bash tools/gpu/ab5.sh $T "--engine-option ensemble_bin_global=0" "--engine-option ensemble_bin_global=1"
