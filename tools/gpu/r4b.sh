# round 4: smoke, the whole -m gpu suite
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r4b}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T.smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/$T.pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$T.pytest_gpu.log; exit $rc
