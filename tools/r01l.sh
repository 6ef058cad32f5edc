cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
VARIANTS=1,2 timeout -k 10 300 python tools/forest_sweep.py > gpurun_out/r01l.sweep.log 2>&1; rc=$?; echo sweep_rc=$rc; tail -5 gpurun_out/r01l.sweep.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 100 --warmup 10 > gpurun_out/r01l.bench2.log 2>&1; rc=$?; echo bench2_rc=$rc; tail -2 gpurun_out/r01l.bench2.log
exit $rc
