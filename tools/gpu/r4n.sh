#!/bin/bash
# round 4: dense card pages behind a 2x key array: smoke, the whole -m gpu suite, config 4 bench
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4n}
[ -z "$SKIP_TESTS" ] && { bash tools/gpu/r4b.sh $T || exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/$T.bench.log 2>&1 || exit $?
grep '^{' gpurun_out/$T.bench.log > gpurun_out/$T.bench.json
python3 -c "import json; d=json.load(open('gpurun_out/$T.bench.json')); print(d['value'], d['ms_per_step'], d['kernel_avg_us'], d['kernel_avg_us_alone'], d['config']['card_pages'])"
