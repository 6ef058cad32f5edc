#!/bin/bash
# one bench line per workload (BASELINE configs + the ingest codec), each under its own limit; JSON lines to
# gpurun_out/T.<workload>.json
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-w}
for W in ${WORKLOADS:-config2 config3 config5 ingest config3j}; do
  timeout -k 10 300 python -u bench.py --workload $W > gpurun_out/$T.$W.log 2>&1 || { echo "$W failed"; exit 1; }
  grep '^{' gpurun_out/$T.$W.log > gpurun_out/$T.$W.json
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], d.get('p99_batch_latency_ms'), (d.get('roofline') or {}).get('kernel_avg_us'), (d.get('roofline') or {}).get('frac'))" gpurun_out/$T.$W.json $W
done
