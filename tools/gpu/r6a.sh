#!/bin/bash
# round 6, first call: the ADVICE / VERDICT test additions (snapshot v2 conversion, config-2 timed kernel, compact
# rows at K = 64), the loopback world sweep, then the gloo rehearsal of `bench.py --gpus 2` and the driver's command
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6a}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_snapshot.py tests/test_gpu_forest.py "tests/test_gpu_pipeline.py::test_pipelined_compact_rows_bit_identical_k64" \
  tests/test_gpu_sharding_loopback.py > gpurun_out/$T.pytest.log 2>&1 || { tail -40 gpurun_out/$T.pytest.log; exit 1; }
tail -3 gpurun_out/$T.pytest.log
FD_BENCH_DIST_BACKEND=gloo timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 20 --warmup 5 --cards 20000000 \
  --no-cpu-baseline > gpurun_out/$T.gloo2.json 2> gpurun_out/$T.gloo2.log || { tail -30 gpurun_out/$T.gloo2.log; exit 1; }
tail -c 1500 gpurun_out/$T.gloo2.json; echo
timeout -k 10 900 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/$T.driver.json 2> gpurun_out/$T.driver.log || { tail -30 gpurun_out/$T.driver.log; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d.get('p99_batch_latency_ms'), d.get('max_batch_latency_ms'), {k: (v.get('value'), v.get('error')) for k, v in (d.get('secondary_workloads') or {}).items()})" gpurun_out/$T.driver.json
