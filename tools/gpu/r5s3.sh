#!/bin/bash
# driver's command: parity oracle before the timed region (old order) vs after it (deferred check), alternating
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s3}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_avg_us']; p=d['parity_vs_oracle']; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], {a[:8]: b for a, b in k.items()}, d.get('diag_blocks_ms_per_step'), p['timed_path']['max_abs_prob_diff'], p['timed_path']['decision_mismatches'], p['twin']['vector_mismatched_elements'])" "$1"; }
for r in 1 2 3; do
  for v in E D; do
    [ $v = E ] && e=1 || e=0
    FD_BENCH_PARITY_EARLY=$e FD_BENCH_BLOCKS=4 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/$T.$v$r.json 2> gpurun_out/$T.$v$r.log || { tail -5 gpurun_out/$T.$v$r.log; exit 1; }
    echo "[$v]"; summ gpurun_out/$T.$v$r.json
  done
done
