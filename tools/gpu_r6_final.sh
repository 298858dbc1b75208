#!/bin/bash
# round 6: full GPU validation + measurement on one box, each step under its own limit, chained so a failing GPU step
# ends the call:  pytest -m gpu, smoke(), bench.py (defaults), rocprofv3 --kernel-trace --stats of bench.py
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${R6_OUT:-r6final}
mkdir -p $O
export TMPDIR=/tmp
set -o pipefail
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { echo "tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
    || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
  tail -3 $O/smoke.txt
fi
timeout -k 10 600 python -u bench.py --full-json $O/bench_full.json ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
tail -n 1 $O/bench.log > $O/bench_line.json
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
      python3 bench.py --no-traffic --no-cpu-baseline --steps 5 --warmup 1 --full-json $O/bench_full_prof.json > $O/prof.log 2>&1 \
    || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
  find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/bench_kernel_stats.csv \;
  # the headline step alone (its gru16p_kernel<5> launches are the roofline's; the full run mixes launch sizes)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_headline -o bench -- \
      python3 bench.py --no-traffic --no-cpu-baseline --no-gru --no-pac --no-conv --no-scl --no-lse --no-mc --steps 5 \
      --warmup 1 --full-json $O/bench_full_headline.json > $O/prof_headline.log 2>&1 || { echo "headline prof failed"; tail -20 $O/prof_headline.log; exit 1; }
  find $O/prof_headline -name "*kernel_stats.csv" -exec cp {} $O/bench_headline_kernel_stats.csv \;
fi
echo "final done"
