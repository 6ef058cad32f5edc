#!/bin/bash
# round 4: the ingest kernel after the word-at-a-time scans — parity tests, per-phase timing, PMC instruction mix
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4e}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ingest.py -m gpu -x -q --timeout 250 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -2 gpurun_out/$T.pytest.log
timeout -k 10 300 python -u tools/ingest_phases.py > gpurun_out/$T.phases.log 2>&1 || exit 1
grep stop_after gpurun_out/$T.phases.log
bash tools/gpu/pmc_ingest.sh $T || exit 1
