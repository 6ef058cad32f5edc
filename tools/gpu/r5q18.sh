#!/bin/bash
# full -m gpu suite, the driver's command twice + a 200-step line, then FETCH / WRITE PMC passes of config 4
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q18}
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_avg_us']; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], d['host_submit_ms_per_step'], {a[:8]: b for a, b in k.items()}, d['parity_vs_oracle']['timed_path']['max_abs_prob_diff'], d['parity_vs_oracle']['timed_path']['decision_mismatches'])" "$1"; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/$T.pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$T.pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$T.pytest_gpu.log
for k in 1 2; do
  timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$T.d$k.json 2> gpurun_out/$T.d$k.log || { tail -20 gpurun_out/$T.d$k.log; exit 1; }
  summ gpurun_out/$T.d$k.json
done
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > gpurun_out/$T.s200.json 2> gpurun_out/$T.s200.log || { tail -20 gpurun_out/$T.s200.log; exit 1; }
summ gpurun_out/$T.s200.json
P4=(--steps 8 --warmup 2 --no-cpu-baseline --latency-iters 2 --loaded-iters 0 --alone-iters 2 --parity-batches 1 --timing-steps 0)
k=0
for p in FETCH_SIZE WRITE_SIZE; do
  k=$((k + 1))
  timeout -s KILL 180 rocprofv3 --pmc $p --output-format csv -d /tmp/$T.c4.p$k -o run -- python bench.py "${P4[@]}" > gpurun_out/$T.c4.p$k.log 2>&1 || { echo "pmc pass $k failed"; exit 1; }
done
python3 tools/pmc_kernels.py config4 65536 ensemble_kernel gpurun_out/$T.pmc_config4_traffic.json /tmp/$T.c4.p* | grep -E "slot_kernel \[grid 65536\]|lean|ensemble_kernel"
