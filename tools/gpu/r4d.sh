# round 4: rocprof stats of the default bench, the native step at world 1, the gloo rehearsal of the N > 1 flow
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4d}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$T.prof -o run -- \
  python bench.py --no-cpu-baseline > gpurun_out/$T.prof.log 2>&1 || exit $?
f=$(find /tmp/$T.prof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/$T.kernel_stats.csv
rm -rf /tmp/$T.prof
VARIANTS=direct,native timeout -k 10 300 python -u tools/route_overhead.py > gpurun_out/$T.route_overhead.log 2>&1 || exit $?
FD_BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --cards 4000000 --steps 20 --warmup 5 \
  --latency-iters 20 --loaded-iters 20 --alone-iters 5 --timing-steps 20 --history-hours 6 --cpu-seconds 1 \
  > gpurun_out/$T.gloo2.log 2>&1
