#!/bin/bash
# fused kernel prologue vs kernel-argument placement: per-wave phases with HIP_FORCE_DEV_KERNARG 0 / 1 / unset
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-s9}
for o in unset 0 1; do
  if [ $o = unset ]; then E=""; else E="HIP_FORCE_DEV_KERNARG=$o"; fi
  env $E CARDS=100000000 STEPS=100 timeout -k 10 400 python3 -u tools/ens_phases_pipe.py > gpurun_out/$T.ens_phases.$o.txt 2> gpurun_out/$T.ens_phases.$o.log || { tail -20 gpurun_out/$T.ens_phases.$o.log; exit 1; }
  echo "== kernarg $o"; grep -A9 "^alone" gpurun_out/$T.ens_phases.$o.txt | grep -E "prologue|total|marks|span"
done
