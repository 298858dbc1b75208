#!/bin/bash
# PMC passes over a child program (one rocprofv3 run per counter group), then a kernel-trace stats run.
#   PMC_CHILD=tools/pmc_gru_child.py PMC_OUT=gpurun_out/pmc_gru bash tools/gpu_pmc_k.sh "CTR CTR ..." ["CTR ..."]
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${PMC_OUT:-gpurun_out/pmck}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o p -- python3 ${PMC_CHILD:-tools/pmc_kernels.py} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o s -- python3 ${PMC_CHILD:-tools/pmc_kernels.py} > $OUT/stats.log 2>&1
echo "stats rc=$?"
