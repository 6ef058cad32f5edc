#!/bin/bash
# (round 5) PMC of the current hot kernels: config 4 (ensemble, slot, lean bucket) and config 5 (lstm_kernel4, split path);
# one rocprofv3 --pmc pass per counter group, each with its own hard limit; summaries -> gpurun_out/T.pmc_*.json
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
export FD_BENCH_SECONDARY=0  # no child workloads under the profiler
T=${1:-pmc}
P4=(--steps 8 --warmup 2 --no-cpu-baseline --latency-iters 2 --loaded-iters 0 --alone-iters 2 --parity-batches 1 --timing-steps 0)
P2=(--workload config2 --steps 8 --warmup 2 --no-cpu-baseline --latency-iters 2 --loaded-iters 0 --alone-iters 2 --parity-batches 1 --timing-steps 0)
P3=(--workload config3 --steps 8 --warmup 2 --no-cpu-baseline --latency-iters 2 --loaded-iters 0 --alone-iters 2 --parity-batches 1 --timing-steps 0)
P5=(--workload config5 --steps 30 --warmup 5 --no-cpu-baseline --latency-iters 2 --loaded-iters 0 --alone-iters 2 --parity-batches 1 --timing-steps 0)
PASSES=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
)
for W in ${WORKLOADS:-4 5}; do
  k=0
  for p in "${PASSES[@]}"; do
    k=$((k + 1))
    if [ $W = 4 ]; then A=("${P4[@]}"); elif [ $W = 3 ]; then A=("${P3[@]}"); elif [ $W = 2 ]; then A=("${P2[@]}"); else A=("${P5[@]}"); fi
    timeout -s KILL 180 rocprofv3 --pmc $p --output-format csv -d /tmp/$T.c$W.p$k -o run -- \
        python bench.py "${A[@]}" > gpurun_out/$T.c$W.p$k.log 2>&1
    rc=$?; echo "config$W pass $k rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
for W in ${WORKLOADS:-4 5}; do
  if [ $W = 4 ]; then python3 tools/pmc_kernels.py config4 65536 ensemble_kernel gpurun_out/$T.pmc_config4.json /tmp/$T.c4.p* || exit $?; fi
  if [ $W = 2 ]; then python3 tools/pmc_kernels.py config2 65536 ensemble_kernel gpurun_out/$T.pmc_config2.json /tmp/$T.c2.p* || exit $?; fi
  if [ $W = 3 ]; then python3 tools/pmc_kernels.py config3 65536 ensemble_kernel gpurun_out/$T.pmc_config3.json /tmp/$T.c3.p* || exit $?; fi
  if [ $W = 5 ]; then python3 tools/pmc_kernels.py config5 1024 lstm_kernel4 gpurun_out/$T.pmc_config5.json /tmp/$T.c5.p* || exit $?; fi
done
rm -rf /tmp/$T.c2.p* /tmp/$T.c3.p* /tmp/$T.c4.p* /tmp/$T.c5.p*
