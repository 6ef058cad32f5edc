#!/bin/bash
# the non-finite W_hh test, then the config-5 workgroup timeline (profiling build) after the pipelined LSTM steps
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s28}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lstm.py \
    > gpurun_out/$T.pytest.txt 2>&1 || { tail -30 gpurun_out/$T.pytest.txt; exit 1; }
tail -2 gpurun_out/$T.pytest.txt
timeout -k 10 300 python3 -u tools/c5_phases.py > gpurun_out/$T.c5_phases.txt 2>&1 || { tail -20 gpurun_out/$T.c5_phases.txt; exit 1; }
cat gpurun_out/$T.c5_phases.txt | tail -25
