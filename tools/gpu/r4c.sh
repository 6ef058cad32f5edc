# round 4: parity of the compact-binning prologue, then config 4 (K = 64) with / without compact vectors, config 5
# with / without the fused latency pair
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4c}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_pipeline.py tests/test_gpu_sharding_loopback.py tests/test_gpu_latency.py tests/test_gpu_ensemble.py \
  tests/test_gpu_configs.py > gpurun_out/$T.pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$T.pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/$T.bench.log 2>&1 || exit $?
grep '^{' gpurun_out/$T.bench.log > gpurun_out/$T.bench.json
timeout -k 10 300 python -u bench.py --engine-option compact_vectors=0 --no-cpu-baseline > gpurun_out/$T.bench_c0.log 2>&1 || exit $?
grep '^{' gpurun_out/$T.bench_c0.log > gpurun_out/$T.bench_c0.json
timeout -k 10 200 python -u bench.py --workload config5 > gpurun_out/$T.config5.log 2>&1 || exit $?
grep '^{' gpurun_out/$T.config5.log > gpurun_out/$T.config5.json
timeout -k 10 200 python -u bench.py --workload config5 --engine-option latency_fused=0 --no-cpu-baseline > gpurun_out/$T.config5_f0.log 2>&1 || exit $?
grep '^{' gpurun_out/$T.config5_f0.log > gpurun_out/$T.config5_f0.json
timeout -k 10 200 python -u bench.py --workload config5 --small-streams 1 --no-cpu-baseline > gpurun_out/$T.config5_s1.log 2>&1 || exit $?
grep '^{' gpurun_out/$T.config5_s1.log > gpurun_out/$T.config5_s1.json
