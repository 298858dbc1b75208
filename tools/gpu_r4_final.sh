#!/bin/bash
# round 4: remaining GPU tests (trained Polar(64,32) fixture, precision), bench line, GRU precision study on the final
# fixture, rocprofv3 kernel stats of the bench, PMC roofline evidence
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "trained_crisp_64_32 or precision" > gpurun_out/pytest_gpu_b.log 2>&1
echo "pytest rc=$?"; grep -E "FAILED|passed|failed" gpurun_out/pytest_gpu_b.log | tail -5
timeout -k 10 420 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log > gpurun_out/bench_line.json
timeout -k 10 300 python -u tools/gru_precision.py --n 65536 --out gpurun_out/gru_precision.json > gpurun_out/gru_precision.log 2>&1; echo "precision rc=$?"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/prof.log 2>&1; echo "rocprof rc=$?"
bash tools/gpu_pmc_r4.sh > gpurun_out/pmc_r4.log 2>&1; echo "pmc rc=$?"
