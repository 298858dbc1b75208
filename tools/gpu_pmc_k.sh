#!/bin/bash
# PMC passes over tools/pmc_kernels.py (one rocprofv3 run per counter group), then a kernel-trace stats run.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmck
export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmck/p$i -o p -- python3 ${PMC_CHILD:-tools/pmc_kernels.py} > gpurun_out/pmck/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmck/p$i.log; exit $rc; fi
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmck/stats -o s -- python3 ${PMC_CHILD:-tools/pmc_kernels.py} > gpurun_out/pmck/stats.log 2>&1
echo "stats rc=$?"
