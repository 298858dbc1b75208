#!/bin/bash
# One GPU session: GRU split-kernel checks + timing, full parity suite, bench line, rocprof stats, co-issue probe.
# Every GPU step has its own time limit; a fault / abort / timeout ends the session.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 0|1) return 0;; *) echo "stopping after rc=$1"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gru_gpu.py tests/test_trained_gru_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gru.log 2>&1
rc=$?; echo "gru pytest rc=$rc"; tail -6 gpurun_out/pytest_gru.log; stop $rc
timeout -k 10 200 python -u tools/gru_prec.py > gpurun_out/gru_prec.log 2>&1
rc=$?; echo "gru_prec rc=$rc"; cat gpurun_out/gru_prec.log; stop $rc
[ -n "$QUICK" ] && exit 0
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; stop $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log; stop $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 2500 gpurun_out/bench.log; stop $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log; stop $rc
timeout -k 10 120 tools/bin/coissue > gpurun_out/coissue.txt 2>&1; echo "coissue rc=$?"; cat gpurun_out/coissue.txt
exit 0
