#!/bin/bash
# PMC of the PAC(128,64) streaming decode under each NPD_SC_ROOT mode (tools/pmc_pac.py as the child)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for m in 1 0; do
  rm -rf gpurun_out/pmck_r$m
  NPD_SC_ROOT=$m PMC_CHILD=tools/pmc_pac.py bash tools/gpu_pmc_k.sh "$@" || exit 1
  mv gpurun_out/pmck gpurun_out/pmck_r$m
done
