#!/bin/bash
# config 5: latency/LSTM/config5 GPU tests, the workgroup timeline (profiling build), the bench line
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-c5c}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_latency.py tests/test_gpu_configs.py tests/test_gpu_lstm.py tests/test_gpu_features.py -k "latency or config5 or lstm or small or fused" > gpurun_out/$T.tests.log 2>&1 || { tail -30 gpurun_out/$T.tests.log; exit 1; }
tail -2 gpurun_out/$T.tests.log
timeout -k 10 300 python -u tools/c5_phases.py > gpurun_out/$T.phases.log 2>&1 || { tail -20 gpurun_out/$T.phases.log; exit 1; }
tail -11 gpurun_out/$T.phases.log
timeout -k 10 300 python -u bench.py --workload config5 --no-cpu-baseline > gpurun_out/$T.bench.log 2>&1 || { tail -20 gpurun_out/$T.bench.log; exit 1; }
grep '^{' gpurun_out/$T.bench.log > gpurun_out/$T.bench.json
python3 -c "import json; d=json.load(open('gpurun_out/$T.bench.json')); print(d['value'], d['ms_per_step'], d['kernel_avg_us'], d['p99_batch_latency_ms'], d['parity_vs_oracle'])"
