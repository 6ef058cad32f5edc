#!/bin/bash
# the fused kernel's compact-row binning: tables staged in LDS (default) vs searched in global memory
# (ensemble_bin_global 1) on the round-6 tree; alternating, the driver's command twice and 200 steps
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6w}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_avg_us']; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], {a[:8]: b for a, b in k.items()}, (d.get('kernel_avg_us_alone') or {}), (d.get('parity_vs_oracle') or {}).get('timed_path', {}).get('max_abs_prob_diff'))" "$1"; }
X="--no-cpu-baseline --loaded-iters 0 --latency-iters 0"
export FD_BENCH_SECONDARY=0
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $X --engine-option ensemble_bin_global=$v > gpurun_out/$T.d$v.$r.json 2> gpurun_out/$T.d$v.$r.log || { tail -5 gpurun_out/$T.d$v.$r.log; exit 1; }
    echo "[20 bin_global=$v]"; summ gpurun_out/$T.d$v.$r.json
  done
done
for v in 0 1; do
  timeout -k 10 300 python3 -u bench.py --steps 200 $X --alone-iters 0 --engine-option ensemble_bin_global=$v > gpurun_out/$T.s$v.json 2> gpurun_out/$T.s$v.log || { tail -5 gpurun_out/$T.s$v.log; exit 1; }
  echo "[200 bin_global=$v]"; summ gpurun_out/$T.s$v.json
done
