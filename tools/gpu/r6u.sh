#!/bin/bash
# slot-stream auto rule from 2^24 slots: pipeline / config tests, then config 3 and 3j with the default
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6u}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d.get('kernel_avg_us'); p=(d.get('parity_vs_oracle') or {}).get('timed_path', {}); print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], k, p.get('max_abs_prob_diff'), p.get('slot_stream_batches'), p.get('decision_mismatches'))" "$1"; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_configs.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
X="--no-cpu-baseline --loaded-iters 0 --alone-iters 0 --latency-iters 0"
for w in config3 config3j; do
  timeout -k 10 400 python3 -u bench.py --workload $w $X > gpurun_out/$T.$w.json 2> gpurun_out/$T.$w.log || { tail -5 gpurun_out/$T.$w.log; exit 1; }
  summ gpurun_out/$T.$w.json
done
