#!/bin/bash
# round 4: ingest structure phase on bit masks: parity, phases, variants, config 3j
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4v}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ingest.py -m gpu -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
timeout -k 10 300 python -u tools/ingest_phases.py > gpurun_out/$T.phases.log 2>&1 || exit 1
grep stop_after gpurun_out/$T.phases.log
timeout -k 10 300 python -u tools/ingest_variants.py base loc_null ts_nofrac > gpurun_out/$T.variants.log 2>&1 || exit 1
grep us gpurun_out/$T.variants.log
timeout -k 10 300 python -u bench.py --workload config3j --no-cpu-baseline > gpurun_out/$T.c3j.log 2>&1 || { tail -20 gpurun_out/$T.c3j.log; exit 1; }
grep '^{' gpurun_out/$T.c3j.log > gpurun_out/$T.c3j.json
python3 -c "import json; d=json.load(open('gpurun_out/$T.c3j.json')); print('c3j', d['value'], d['ms_per_step'], d['kernel_avg_us'], d['parity_vs_oracle']['decision_mismatches'])"
