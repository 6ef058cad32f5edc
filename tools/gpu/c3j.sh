#!/bin/bash
# config 3j: the fused kernel's chunk layout (wide 148 KB LDS vs compact 132 KB: room for an ingest workgroup beside)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-c3j}
for V in 0 1; do
  timeout -k 10 400 python -u bench.py --workload config3j --no-cpu-baseline --engine-option ingest_prio=$V > gpurun_out/$T.$V.log 2>&1 || { tail -20 gpurun_out/$T.$V.log; exit 1; }
  grep '^{' gpurun_out/$T.$V.log > gpurun_out/$T.$V.json
  python3 -c "import json; d=json.load(open('gpurun_out/$T.$V.json')); p=d['parity_vs_oracle']; print('prio=$V', d['value'], d['ms_per_step'], d['kernel_avg_us'], {k: p.get(k) for k in ('vector_mismatched_elements','max_abs_prob_diff','decision_mismatches','columns_mismatched')})"
done
timeout -k 10 300 python -u bench.py --workload ingest --no-cpu-baseline > gpurun_out/$T.ingest.log 2>&1 || { tail -20 gpurun_out/$T.ingest.log; exit 1; }
grep '^{' gpurun_out/$T.ingest.log > gpurun_out/$T.ingest.json
python3 -c "import json; d=json.load(open('gpurun_out/$T.ingest.json')); print('ingest alone', d['value'], d['ms_per_step'], d.get('parity_vs_oracle'))"
