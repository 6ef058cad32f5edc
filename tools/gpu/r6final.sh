#!/bin/bash
# round 6 evidence on the current tree: smoke + the whole -m gpu suite, the driver's own bench command
# (--steps 20 --warmup 5) twice, the default 200-step line, and the driver command under rocprofv3 --kernel-trace --stats
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-fin}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); p=d.get('parity_vs_oracle') or {}; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], d.get('p99_batch_latency_ms'), d.get('max_batch_latency_ms'), d['kernel_avg_us'], json.dumps(p.get('timed_path')), {k: v.get('value') for k, v in (d.get('secondary_workloads') or {}).items()})" "$1"; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T.smoke.log 2>&1 || { tail -20 gpurun_out/$T.smoke.log; exit 1; }
tail -1 gpurun_out/$T.smoke.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$T.pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$T.pytest_gpu.log
for k in 1 2; do
  timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$T.d$k.json 2> gpurun_out/$T.d$k.log || { tail -20 gpurun_out/$T.d$k.log; exit 1; }
  summ gpurun_out/$T.d$k.json
done
FD_BENCH_SECONDARY=0 timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > gpurun_out/$T.s200.json 2> gpurun_out/$T.s200.log || { tail -20 gpurun_out/$T.s200.log; exit 1; }
summ gpurun_out/$T.s200.json
FD_BENCH_SECONDARY=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$T.prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$T.prof.log 2>&1 || { tail -20 gpurun_out/$T.prof.log; exit 1; }
mkdir -p gpurun_out/$T.prof
find /tmp/$T.prof -name '*stats.csv' -exec cp {} gpurun_out/$T.prof/ \;
grep '^{' gpurun_out/$T.prof.log > gpurun_out/$T.prof_bench.json
summ gpurun_out/$T.prof_bench.json
