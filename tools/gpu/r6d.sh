#!/bin/bash
# host cost of the native sharded step at world 1 (self share as a device copy), then the driver's command with the
# per-sample latency split
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6d}
VARIANTS=direct,native STEPS=200 timeout -k 10 500 python3 -u tools/route_overhead.py > gpurun_out/$T.route.txt 2> gpurun_out/$T.route.log || { tail -20 gpurun_out/$T.route.log; exit 1; }
cat gpurun_out/$T.route.txt
timeout -k 10 900 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/$T.driver.json 2> gpurun_out/$T.driver.log || { tail -30 gpurun_out/$T.driver.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['p99_batch_latency_ms'], d['max_batch_latency_ms'], json.dumps(d.get('latency_split')), json.dumps({k: d['loaded_latency'][k] for k in ('p50_ms','p99_ms','max_ms','worst','host_submit_ms_max')}), {k: (v.get('value'), v.get('error')) for k, v in (d.get('secondary_workloads') or {}).items()})" gpurun_out/$T.driver.json
