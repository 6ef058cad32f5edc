#!/bin/bash
# xwide layout (ensemble_chunks 3: 28 trees per chunk, TPG 7) vs wide (1): parity tests, per-wave phases, alone + pipelined
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s4}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ensemble.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$T.pytest_ens.log 2>&1 || { tail -40 gpurun_out/$T.pytest_ens.log; exit 1; }
tail -1 gpurun_out/$T.pytest_ens.log
for o in 3 1; do
  OPTS=ensemble_chunks=$o CARDS=100000000 STEPS=200 timeout -k 10 400 python3 -u tools/ens_phases_pipe.py > gpurun_out/$T.ens_phases.$o.txt 2> gpurun_out/$T.ens_phases.$o.log || { tail -20 gpurun_out/$T.ens_phases.$o.log; exit 1; }
  echo "== chunks $o"; cat gpurun_out/$T.ens_phases.$o.txt
done
for r in 1 2; do
for o in 1 3; do
  timeout -k 10 300 python3 -u bench.py --steps 200 --no-cpu-baseline --loaded-iters 0 --latency-iters 0 --engine-option ensemble_chunks=$o > gpurun_out/$T.c$o.$r.json 2> gpurun_out/$T.c$o.$r.log || { tail -5 gpurun_out/$T.c$o.$r.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], r['kernel_avg_us'], r['frac'], r['alone'], d['parity_vs_oracle']['timed_path']['max_abs_prob_diff'])" gpurun_out/$T.c$o.$r.json
done
done
