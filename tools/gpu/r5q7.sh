#!/bin/bash
# is the slow start the batches (which resident micro-batches the region uses) or what ran before it?
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q7}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], d.get('diag_blocks_ms_per_step'))" "$1"; }
B="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --loaded-iters 0 --alone-iters 0"
FD_BENCH_LATENCY_FIRST=0 FD_BENCH_BLOCKS=8 FD_BENCH_BATCH_OFFSET=400 timeout -k 10 400 python3 -u bench.py $B > gpurun_out/$T.off.json 2> gpurun_out/$T.off.log || exit 1
summ gpurun_out/$T.off.json
FD_BENCH_LATENCY_FIRST=0 FD_BENCH_BLOCKS=8 timeout -k 10 400 python3 -u bench.py $B > gpurun_out/$T.base.json 2> gpurun_out/$T.base.log || exit 1
summ gpurun_out/$T.base.json
FD_BENCH_LATENCY_FIRST=0 FD_BENCH_BLOCKS=8 timeout -k 10 400 python3 -u bench.py $B --latency-iters 0 > gpurun_out/$T.nolat.json 2> gpurun_out/$T.nolat.log || exit 1
summ gpurun_out/$T.nolat.json
