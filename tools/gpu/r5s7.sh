#!/bin/bash
# round-close style check of the current tree: smoke + full -m gpu suite + the driver's command (with its secondary
# workloads) + a 200-step line + rocprofv3 kernel-trace stats of the driver's command (secondaries off)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s7}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T.smoke.log 2>&1 || { tail -20 gpurun_out/$T.smoke.log; exit 1; }
tail -1 gpurun_out/$T.smoke.log
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$T.pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$T.pytest_gpu.log
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$T.d.json 2> gpurun_out/$T.d.log || { tail -20 gpurun_out/$T.d.log; exit 1; }
FD_BENCH_SECONDARY=0 timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > gpurun_out/$T.s200.json 2> gpurun_out/$T.s200.log || { tail -20 gpurun_out/$T.s200.log; exit 1; }
for f in d s200; do python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']
print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], d['host_submit_ms_per_step'], r['kernel_avg_us'], r['frac'], r['alone'], r['attainable']['frac'], d['parity_vs_oracle']['timed_path']['max_abs_prob_diff'], d['p99_batch_latency_ms'])
for k,v in (d.get('secondary_workloads') or {}).items(): print('  ', k, v.get('value'), v.get('ms_per_step'), v.get('p99_batch_latency_ms'), (v.get('roofline') or {}).get('frac'))
" gpurun_out/$T.$f.json; done
FD_BENCH_SECONDARY=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$T.prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$T.prof.log 2>&1 || { tail -20 gpurun_out/$T.prof.log; exit 1; }
cp "$(find /tmp/$T.prof -name "*kernel_stats.csv" | head -1)" gpurun_out/$T.prof_kernel_stats.csv && echo "kernel stats -> gpurun_out/$T.prof_kernel_stats.csv"
