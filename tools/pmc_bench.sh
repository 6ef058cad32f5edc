#!/bin/bash
# HBM-traffic PMC passes over bench.py (one TCC counter group per pass, --kernel-trace only, as
# MI355X_MICROARCH.md "rocprofv3 PMC slots" prescribes), then tools/pmc_summarize.py writes
# profiles/pmc_<workload>.json (hbm_bytes_per_launch of the dominant kernel, gfx950-corrected).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-pmc}; WL=${WL:-config2}; EXTRA=${EXTRA:-}
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/$TAG.$WL.p$i -o run -- \
     python bench.py --workload $WL --steps 20 --warmup 3 --latency-iters 0 --no-cpu-baseline $EXTRA \
     > gpurun_out/$TAG.$WL.p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python tools/pmc_summarize.py gpurun_out/$TAG.$WL $WL
# profiles/pmc_<wl>.json is written on the box (not merged back): re-run tools/pmc_summarize.py here on gpurun_out/
