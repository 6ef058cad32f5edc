#!/bin/bash
# (round 5) instruction / scalar cache counters of the config-4 kernels: is the fused kernel's ~27k-cycle prologue
# instruction-fetch bound (50 KB of code per instantiation, the four thread-quarter paths unrolled)?
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
export FD_BENCH_SECONDARY=0
T=${1:-s25}
P4=(--steps 8 --warmup 2 --no-cpu-baseline --latency-iters 2 --loaded-iters 0 --alone-iters 2 --parity-batches 1 --timing-steps 0)
PASSES=(
  "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES SQ_WAVES"
  "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_INSTS_SALU"
)
k=0
for p in "${PASSES[@]}"; do
  k=$((k + 1))
  timeout -s KILL 150 rocprofv3 --pmc $p --output-format csv -d /tmp/$T.p$k -o run -- \
      python bench.py "${P4[@]}" > gpurun_out/$T.p$k.log 2>&1
  rc=$?; echo "pass $k rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/$T.p$k.log; exit $rc; }
done
python3 tools/pmc_kernels.py config4 65536 ensemble_kernel gpurun_out/$T.pmc_icache.json /tmp/$T.p* || exit $?
rm -rf /tmp/$T.p*
