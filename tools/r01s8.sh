cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/s8; export TMPDIR=/tmp
O=gpurun_out/s8
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo smoke_rc=$rc; tail -1 $O/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $O/bench_config2.json.log 2>&1; rc=$?; echo c2_rc=$rc; tail -1 $O/bench_config2.json.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --workload ingest --steps 100 --warmup 10 --cpu-seconds 8 --latency-iters 50 > $O/bench_ingest.json.log 2>&1; rc=$?; echo ing_rc=$rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ingprof -o run -- python bench.py --workload ingest --steps 30 --warmup 5 --no-cpu-baseline --latency-iters 5 > $O/ingprof.log 2>&1; rc=$?; echo ingprof_rc=$rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py --workload config3j --steps 100 --warmup 10 --cpu-seconds 8 --latency-iters 100 > $O/bench_config3j.json.log 2>&1; rc=$?; echo c3j_rc=$rc; tail -1 $O/bench_config3j.json.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3jprof -o run -- python bench.py --workload config3j --steps 30 --warmup 5 --no-cpu-baseline --latency-iters 5 > $O/c3jprof.log 2>&1; rc=$?; echo c3jprof_rc=$rc
exit $rc
