#!/bin/bash
# PMC passes over a short bench run (each counter group in its own rocprofv3 run; no tracing domains).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline --no-gru"}
[ -n "$LIST" ] && (rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1; echo "list rc=$?")
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/p$i -o p -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/p$i.log; exit $rc; fi
done
