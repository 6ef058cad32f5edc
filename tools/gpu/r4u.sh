#!/bin/bash
# round 4: ingest at two waves per workgroup (19.5 KB LDS): parity, alone, config 3j pipelined with the compact
# ensemble layout (room on the CU for a codec workgroup) and with the wide one
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4u}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ingest.py -m gpu -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
timeout -k 10 300 python -u tools/ingest_phases.py 0 > gpurun_out/$T.phases.log 2>&1 || exit 1
grep stop_after gpurun_out/$T.phases.log
for V in "--engine-option ensemble_chunks=2" ""; do
  N=$(echo "x$V" | tr -d ' -=')
  timeout -k 10 300 python -u bench.py --workload config3j --no-cpu-baseline $V > gpurun_out/$T.$N.log 2>&1 || { tail -20 gpurun_out/$T.$N.log; exit 1; }
  grep '^{' gpurun_out/$T.$N.log > gpurun_out/$T.$N.json
  python3 -c "import json; d=json.load(open('gpurun_out/$T.$N.json')); print('$V', d['value'], d['ms_per_step'], d['p99_batch_latency_ms'], d['kernel_avg_us'], d['parity_vs_oracle']['decision_mismatches'])"
done
