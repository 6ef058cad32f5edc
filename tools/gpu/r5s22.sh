#!/bin/bash
# bucket size under the lean kernel at priority 2: bucket_keys 64 / auto (128) / 256, 200 steps, two rounds
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s22}
export FD_BENCH_SECONDARY=0
X="--no-cpu-baseline --loaded-iters 0 --latency-iters 0"
for r in 1 2; do
  for v in 64 0 256; do
    timeout -k 10 300 python3 -u bench.py --steps 200 $X --engine-option bucket_keys=$v > gpurun_out/$T.k$v.$r.json 2> gpurun_out/$T.k$v.$r.log || { tail -5 gpurun_out/$T.k$v.$r.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_avg_us']; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], {a[:8]: b for a, b in k.items()})" gpurun_out/$T.k$v.$r.json
  done
done
