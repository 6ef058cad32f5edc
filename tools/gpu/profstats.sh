#!/bin/bash
# the default bench under rocprofv3 --kernel-trace --stats: keep only the stats summaries (the trace is large)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-profstats}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$T.prof -o run -- python3 -u bench.py --no-cpu-baseline > gpurun_out/$T.prof.log 2>&1 || { tail -20 gpurun_out/$T.prof.log; exit 1; }
du -a /tmp/$T.prof | sort -n | tail -8
mkdir -p gpurun_out/$T.prof
find /tmp/$T.prof -name '*stats.csv' -exec cp {} gpurun_out/$T.prof/ \;
grep '^{' gpurun_out/$T.prof.log > gpurun_out/$T.prof_bench.json
ls -la gpurun_out/$T.prof
