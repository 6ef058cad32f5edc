#!/bin/bash
# every workload's bench line on the current tree (builder-run), the driver's step/warmup counts
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q15}
for W in config5 config3 config2 ingest config3j; do
  timeout -k 10 300 python3 -u bench.py --workload $W --steps 20 --warmup 5 > gpurun_out/$T.$W.json 2> gpurun_out/$T.$W.log || { echo "$W failed"; tail -5 gpurun_out/$T.$W.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); p=d.get('parity_vs_oracle') or {}; r=d.get('roofline') or {}; print(sys.argv[2], round(d['value']/1e6,2), d['ms_per_step'], d.get('p99_batch_latency_ms'), r.get('kernel_avg_us'), r.get('frac'), d['kernel_avg_us'], json.dumps(p)[:300])" gpurun_out/$T.$W.json $W
done
for W in config5 config3; do
  timeout -k 10 300 python3 -u bench.py --workload $W --no-cpu-baseline > gpurun_out/$T.${W}_200.json 2> gpurun_out/$T.${W}_200.log || { echo "$W failed"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '200 steps', round(d['value']/1e6,2), d['ms_per_step'], d['kernel_avg_us'])" gpurun_out/$T.${W}_200.json $W
done
