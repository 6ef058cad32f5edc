#!/bin/bash
# round 4: config 4 features vs the card table's load factor (K = 16 at r03's 1.6 slots per card; K = 64 at 1.25),
# rocprof kernel stats of the default bench
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4h}
timeout -k 10 300 python -u bench.py --no-cpu-baseline --ring-k 16 --slots-per-card 1.6 > gpurun_out/$T.k16s16.log 2>&1 || exit $?
grep '^{' gpurun_out/$T.k16s16.log > gpurun_out/$T.k16s16.json
python3 -c "import json; d=json.load(open('gpurun_out/$T.k16s16.json')); print(d['value'], d['ms_per_step'], d['kernel_avg_us'], d['kernel_avg_us_alone'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$T.prof -o run -- \
  python bench.py --no-cpu-baseline > gpurun_out/$T.prof.log 2>&1 || exit $?
f=$(find /tmp/$T.prof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/$T.kernel_stats.csv
rm -rf /tmp/$T.prof
