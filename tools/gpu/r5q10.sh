#!/bin/bash
# lean bucket kernel phases in the pipeline (profiling library), world 8 over the loopback, host phases per world
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q10}
FDENGINE_LIB=$PWD/realtime-fraud-detection_amd/lib/libfdengine_prof.so FD_BENCH_DUMP_FPROF=gpurun_out/$T.fp FD_BENCH_BLOCKS=8 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --loaded-iters 0 --alone-iters 0 --latency-iters 0 > gpurun_out/$T.prof.json 2> gpurun_out/$T.prof.log || { tail -5 gpurun_out/$T.prof.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$T.prof.json')); print(d['ms_per_step'], d.get('diag_blocks_ms_per_step'))"
python3 tools/lean_phases.py gpurun_out/$T.fp.*.npy | tee gpurun_out/$T.lean_phases.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharding_loopback.py -x -v --timeout 300 --timeout-method thread > gpurun_out/$T.loopback.log 2>&1 || { tail -30 gpurun_out/$T.loopback.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/$T.loopback.log | tail -12
timeout -k 10 600 python3 -u tools/loopback_host.py 1,2,4,8 16384 40 > gpurun_out/$T.lbhost.json 2> gpurun_out/$T.lbhost.log || { tail -20 gpurun_out/$T.lbhost.log; exit 1; }
head -4 gpurun_out/$T.lbhost.json
