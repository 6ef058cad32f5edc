#!/bin/bash
# binning tables staged by LDS-DMA from per-plan padded images: parity subset, per-wave phases, driver command x2 + 200
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q20}
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_configs.py tests/test_gpu_ensemble.py tests/test_gpu_forest.py -x -v --timeout 300 --timeout-method thread > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
CARDS=100000000 STEPS=200 timeout -k 10 400 python3 -u tools/ens_phases_pipe.py > gpurun_out/$T.ens_phases.txt 2> gpurun_out/$T.ens_phases.log || { tail -20 gpurun_out/$T.ens_phases.log; exit 1; }
cat gpurun_out/$T.ens_phases.txt
bash tools/gpu/ab5.sh $T "" "--engine-option ensemble_int_lut=1"
