#!/bin/bash
# Round-2 GPU session: selected parity tests (TESTS), the bench (BENCH_ARGS), optional rocprof kernel stats.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest.log | tail -15
  [ $rc -ne 0 ] && exit $rc
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 4000 gpurun_out/bench.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof -name "*stats*"
  exit $rc
fi
exit 0
