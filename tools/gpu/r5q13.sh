#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-q13}
FDENGINE_LIB=$PWD/realtime-fraud-detection_amd/lib/libfdengine_prof.so FD_BENCH_DUMP_FPROF=gpurun_out/$T.fp FD_BENCH_BLOCKS=2 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --loaded-iters 0 --alone-iters 0 --latency-iters 0 > gpurun_out/$T.prof.json 2> gpurun_out/$T.prof.log || { tail -5 gpurun_out/$T.prof.log; exit 1; }
python3 tools/lean_phases.py gpurun_out/$T.fp.*.npy | tee gpurun_out/$T.lean_phases.txt
