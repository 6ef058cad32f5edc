#!/bin/bash
# config 5 pipelined with the gather bucket kernel (option pipeline_gather) against the one-stream default and the
# pipelined slot + lean pair; the pipeline parity tests first
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s26}
export FD_BENCH_SECONDARY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    "tests/test_gpu_pipeline.py::test_pipelined_lstm_and_latency_batches" tests/test_gpu_latency.py \
    > gpurun_out/$T.pytest.txt 2>&1 || { tail -30 gpurun_out/$T.pytest.txt; exit 1; }
tail -2 gpurun_out/$T.pytest.txt
for r in 1 2; do
  for v in serial pg1 pg0; do
    case $v in
      serial) A=() ;;
      pg1) A=(--pipeline --engine-option pipeline_gather=1) ;;
      pg0) A=(--pipeline --engine-option pipeline_gather=0) ;;
    esac
    timeout -k 10 300 python3 -u bench.py --workload config5 --steps 200 --no-cpu-baseline "${A[@]}" > gpurun_out/$T.$v.$r.json 2> gpurun_out/$T.$v.$r.log || { tail -5 gpurun_out/$T.$v.$r.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,2), d['ms_per_step'], d['p99_batch_latency_ms'], d['kernel_avg_us'], d.get('parity_vs_oracle',{}).get('timed_path'))" gpurun_out/$T.$v.$r.json
  done
done
