#!/bin/bash
# LSE parity first (new kernel), then the whole GPU suite, the bench and rocprof kernel stats.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_lse_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_lse.log 2>&1
rc=$?; echo "lse pytest rc=$rc"; tail -15 gpurun_out/pytest_lse.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "gpu pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof -name "*stats*"
exit $rc
