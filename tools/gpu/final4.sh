#!/bin/bash
# round 4 close: smoke, the whole -m gpu suite, the default bench line (rocprof stats: tools/gpu/profstats.sh)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-final4}
bash tools/gpu/r4b.sh $T || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/$T.bench.log 2>&1 || { tail -20 gpurun_out/$T.bench.log; exit 1; }
grep '^{' gpurun_out/$T.bench.log > gpurun_out/$T.bench.json
python3 -c "import json; d=json.load(open('gpurun_out/$T.bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['p99_batch_latency_ms'], d.get('p99_batch_latency_with_h2d_ms'), d['parity_vs_oracle'])"
bash tools/gpu/profstats.sh $T
