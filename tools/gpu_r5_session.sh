#!/bin/bash
# round 5 GPU session: optional steps chosen by environment variables, each under its own time limit, chained so
# that a failing GPU step ends the call (training runs last, in the remaining budget).
#   GAP=1           tools/bin/gapbench (MFMA gap-filling cost model)
#   AB="a.so b.so"  tools/gru16_time.py A/B of libnpd builds (fp16x3 GRU, trained net)
#   CONV_AB="a.so b.so"  tools/conv_time.py per library (configs[4] conv forward, fp32 and fp16x3)
#   TESTS="k expr"  pytest -m gpu -k expr
#   BENCH=1         bench.py (default flags) -> gpurun_out/bench_r5.json / .log
#   PROF=1          rocprofv3 --kernel-trace --stats of bench.py
#   TRAIN=seconds   one slice of the Polar(64,22) hidden-512 curriculum
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
set -o pipefail
if [ -n "$GAP" ]; then
  timeout -k 10 120 tools/bin/gapbench > gpurun_out/gapbench.txt 2>&1 || { echo "gapbench failed"; exit 1; }
  cat gpurun_out/gapbench.txt
fi
if [ -n "$AB" ]; then
  timeout -k 10 600 python -u tools/gru16_time.py $AB --rounds ${AB_ROUNDS:-2} > gpurun_out/gru16_ab.txt 2>&1 \
    || { echo "A/B failed"; tail -20 gpurun_out/gru16_ab.txt; exit 1; }
  cat gpurun_out/gru16_ab.txt
fi
if [ -n "$CONV_AB" ]; then
  for lib in $CONV_AB; do
    echo "== $lib" >> gpurun_out/conv_ab.txt
    NPD_LIB=$(readlink -f $lib) timeout -k 10 300 python -u tools/conv_time.py 2 >> gpurun_out/conv_ab.txt 2>&1 \
      || { echo "conv A/B failed"; tail -20 gpurun_out/conv_ab.txt; exit 1; }
  done
  cat gpurun_out/conv_ab.txt
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$TESTS" \
    > gpurun_out/pytest_r5.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_r5.log; exit 1; }
  tail -3 gpurun_out/pytest_r5.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_r5.log 2>&1 \
    || { echo "bench failed"; tail -30 gpurun_out/bench_r5.log; exit 1; }
  tail -n 1 gpurun_out/bench_r5.log > gpurun_out/bench_r5.json
  cat gpurun_out/bench_r5.json
fi
if [ -n "$PROF" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r5 -o run -- python3 bench.py --full-json gpurun_out/bench_full_prof.json --no-traffic \
    --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/prof_r5.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_r5.log; exit 1; }
  find gpurun_out/prof_r5 -name "*kernel_stats.csv" | head -3
fi
if [ -n "$TRAIN" ]; then
  BUDGET=$TRAIN bash tools/gpu_r5_train.sh
fi
exit 0
