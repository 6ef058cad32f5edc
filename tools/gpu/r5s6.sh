#!/bin/bash
# the driver's command with the secondary workloads (config 5 / 2 / 3 as child processes), timed
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s6}
a=$(date +%s.%N)
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$T.d.json 2> gpurun_out/$T.d.log || { tail -20 gpurun_out/$T.d.log; exit 1; }
b=$(date +%s.%N)
python3 -c "import sys; print('wall', round(float(sys.argv[2]) - float(sys.argv[1]), 1), 's')" $a $b
python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(round(d['value']/1e6,1), d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('attainable'))
for k,v in (d.get('secondary_workloads') or {}).items(): print(k, json.dumps(v)[:900])
" gpurun_out/$T.d.json
