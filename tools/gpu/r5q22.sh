#!/bin/bash
# ensemble_dma_rot A/B: per-wave phases for 0 / 1 / 2 on one box, then the driver command 0 vs 1
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q22}
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
for o in 0 1 2 0; do
  OPTS=ensemble_dma_rot=$o CARDS=100000000 STEPS=200 timeout -k 10 400 python3 -u tools/ens_phases_pipe.py > gpurun_out/$T.ens_phases.$o.txt 2> gpurun_out/$T.ens_phases.$o.log || { tail -20 gpurun_out/$T.ens_phases.$o.log; exit 1; }
  echo "== rot $o"; grep -E "total|prologue  |marks|walk\+leaf by|span" gpurun_out/$T.ens_phases.$o.txt
done
bash tools/gpu/ab5.sh $T "--engine-option ensemble_dma_rot=0" "--engine-option ensemble_dma_rot=1"
