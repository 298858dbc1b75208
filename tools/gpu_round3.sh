#!/bin/bash
# Round-3 GPU session: parity tests, full bench line, rocprof kernel stats of the bench.  Stops at the first fault/timeout.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
fi
exit 0
