#!/bin/bash
# config 5: fd_score_batch_device per step (default) vs the pipelined stream (--pipeline), alternating
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s12}
for r in 1 2; do
  for v in D P; do
    [ $v = P ] && o="--pipeline" || o=""
    FD_BENCH_SECONDARY=0 timeout -k 10 300 python3 -u bench.py --workload config5 --steps 200 --warmup 20 --no-cpu-baseline $o > gpurun_out/$T.$v$r.json 2> gpurun_out/$T.$v$r.log || { tail -5 gpurun_out/$T.$v$r.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); p=d['parity_vs_oracle']; print(sys.argv[1], round(d['value']/1e6,2), d['ms_per_step'], d['host_submit_ms_per_step'], d['p99_batch_latency_ms'], d['kernel_avg_us'], {k: v for k, v in p.items() if 'diff' in k or 'mismatch' in k})" gpurun_out/$T.$v$r.json
  done
done
