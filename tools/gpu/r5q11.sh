#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q11}
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_configs.py tests/test_gpu_features_segments.py tests/test_gpu_sharding_loopback.py -x -v --timeout 300 --timeout-method thread > gpurun_out/$T.pytest.log 2>&1 || { tail -30 gpurun_out/$T.pytest.log; exit 1; }
tail -1 gpurun_out/$T.pytest.log
FDENGINE_LIB=$PWD/realtime-fraud-detection_amd/lib/libfdengine_prof.so FD_BENCH_DUMP_FPROF=gpurun_out/$T.fp FD_BENCH_BLOCKS=2 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --loaded-iters 0 --alone-iters 0 --latency-iters 0 > gpurun_out/$T.prof.json 2> gpurun_out/$T.prof.log || { tail -5 gpurun_out/$T.prof.log; exit 1; }
python3 tools/lean_phases.py gpurun_out/$T.fp.*.npy | tee gpurun_out/$T.lean_phases.txt
bash tools/gpu/ab5.sh $T "--engine-option lean_group=1" "--engine-option lean_group=2"
