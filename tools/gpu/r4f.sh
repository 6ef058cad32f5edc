#!/bin/bash
# round 4: ingest after the word scans (tests, phases, variants, PMC); config 4's features at ring_k 16 / 32 / 64;
# then r4d (rocprof stats, route overhead, gloo rehearsal)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4f}
bash tools/gpu/r4e.sh $T || exit 1
timeout -k 10 300 python -u tools/ingest_variants.py > gpurun_out/$T.variants.log 2>&1 || exit 1
cat gpurun_out/$T.variants.log | grep us
for K in 16 32; do
  timeout -k 10 300 python -u bench.py --ring-k $K --no-cpu-baseline > gpurun_out/$T.bench_k$K.log 2>&1 || exit $?
  grep '^{' gpurun_out/$T.bench_k$K.log > gpurun_out/$T.bench_k$K.json
done
bash tools/gpu/r4d.sh $T
