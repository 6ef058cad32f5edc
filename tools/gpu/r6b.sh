#!/bin/bash
# split rows (compact_vectors 2): parity (pipeline twin tests, config-4 full size, loopback), HBM traffic of the
# feature kernels for compact 64-B rows vs split rows (FETCH / WRITE passes), then the A/B on the driver's command
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6b}
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_pipeline.py tests/test_gpu_configs.py tests/test_gpu_golden_full.py \
  tests/test_gpu_sharding_loopback.py \
  > gpurun_out/$T.pytest.log 2>&1 || { tail -40 gpurun_out/$T.pytest.log; exit 1; }
tail -3 gpurun_out/$T.pytest.log
export FD_BENCH_SECONDARY=0
P4=(--steps 8 --warmup 2 --no-cpu-baseline --latency-iters 2 --loaded-iters 0 --alone-iters 2 --parity-batches 1 --timing-steps 0)
for cv in 1 2; do
  k=0
  for p in FETCH_SIZE WRITE_SIZE; do
    k=$((k + 1))
    timeout -s KILL 180 rocprofv3 --pmc $p --output-format csv -d /tmp/$T.cv$cv.p$k -o run -- \
        python bench.py "${P4[@]}" --engine-option compact_vectors=$cv > gpurun_out/$T.cv$cv.p$k.log 2>&1
    rc=$?; echo "compact_vectors $cv pass $k rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
  python3 tools/pmc_kernels.py config4 65536 ensemble_kernel gpurun_out/$T.pmc_cv$cv.json /tmp/$T.cv$cv.p* || exit $?
done
rm -rf /tmp/$T.cv*
unset FD_BENCH_SECONDARY
bash tools/gpu/ab5.sh $T "--engine-option compact_vectors=1" "--engine-option compact_vectors=2"
