# round 4: the N>=2 native step over the RCCL loopback, the segment / ensemble parity tests, then the A/B of the
# scalar top-level walk
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sharding_loopback.py \
  tests/test_gpu_sharding.py tests/test_gpu_ensemble.py tests/test_gpu_pipeline.py tests/test_gpu_latency.py tests/test_gpu_features_segments.py > gpurun_out/r4a.pytest.log 2>&1 &&
OPTS="ensemble_scalar_top=0;ensemble_scalar_top=1" ROUNDS=8 timeout -k 10 300 python -u tools/ens_ab.py > gpurun_out/r4a.ens_ab.log 2>&1
