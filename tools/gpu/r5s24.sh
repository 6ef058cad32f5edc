#!/bin/bash
# config 5 knobs re-measured on the final tree: small_streams 0 (default) / 1 / 2, two rounds, 200 steps
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s24}
export FD_BENCH_SECONDARY=0
for r in 1 2; do
  for v in 0 1 2; do
    timeout -k 10 300 python3 -u bench.py --workload config5 --steps 200 --no-cpu-baseline --small-streams $v > gpurun_out/$T.ss$v.$r.json 2> gpurun_out/$T.ss$v.$r.log || { tail -5 gpurun_out/$T.ss$v.$r.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,2), d['ms_per_step'], d['p99_batch_latency_ms'], d['kernel_avg_us'])" gpurun_out/$T.ss$v.$r.json
  done
done
