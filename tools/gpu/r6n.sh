#!/bin/bash
# lean bucket kernel phases in the pipeline (profiling build), default priorities, then feature_prio 1 for contrast
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r6n}
X="--no-cpu-baseline --loaded-iters 0 --latency-iters 0 --alone-iters 0 --timing-steps 0"
export FD_BENCH_SECONDARY=0 FDENGINE_LIB=$PWD/realtime-fraud-detection_amd/lib/libfdengine_prof.so
for o in "" "--engine-option feature_prio=1"; do
  tag=$([ -z "$o" ] && echo def || echo fp1)
  FD_BENCH_DUMP_FPROF=gpurun_out/$T.$tag timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $X $o > gpurun_out/$T.$tag.json 2> gpurun_out/$T.$tag.log || { tail -5 gpurun_out/$T.$tag.log; exit 1; }
  echo "== $tag $o"; python3 tools/lean_phases.py gpurun_out/$T.$tag.*.npy 2>&1 | tail -14
done
