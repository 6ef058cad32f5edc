#!/bin/bash
# SQ instruction-mix PMC pass over the ingest bench (one pass, 8 SQ counters, --kernel-trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM \
  --kernel-trace --output-format csv -d gpurun_out/sqing -o run -- \
  python bench.py --workload ingest --steps 10 --warmup 2 --latency-iters 0 --no-cpu-baseline > gpurun_out/sqing.log 2>&1
rc=$?; echo "sq pass rc=$rc"; exit $rc
