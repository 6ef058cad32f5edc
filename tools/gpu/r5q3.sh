#!/bin/bash
# the driver's command after the bench reorder (latency loops before the throughput region), three times, with the
# per-block rates after it
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q3}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], d['host_submit_ms_per_step'], (d.get('host_submit_breakdown') or {}).get('native_us_per_step'), d.get('p99_batch_latency_ms'), d.get('p99_batch_latency_with_h2d_ms'), d.get('diag_blocks_ms_per_step'))" "$1"; }
for k in 1 2 3; do
  FD_BENCH_BLOCKS=4 timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$T.d$k.json 2> gpurun_out/$T.d$k.log || { tail -20 gpurun_out/$T.d$k.log; exit 1; }
  summ gpurun_out/$T.d$k.json
done
FD_BENCH_BLOCKS=2 timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > gpurun_out/$T.s200.json 2> gpurun_out/$T.s200.log || { tail -20 gpurun_out/$T.s200.log; exit 1; }
summ gpurun_out/$T.s200.json
