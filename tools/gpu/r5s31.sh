#!/bin/bash
# the driver's short region vs long runs on the device's own clocks (tools/clock_ramp.py, profiling build):
# shader clock and launch-to-launch step time per 20-launch block, after 3 s / 0 s of host-only time
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s31}
for idle in 3 0; do
  IDLE=$idle STEPS=200 timeout -k 10 400 python3 -u tools/clock_ramp.py > gpurun_out/$T.idle$idle.txt 2>&1 || { tail -20 gpurun_out/$T.idle$idle.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/$T.idle$idle.txt | tail -14
done
