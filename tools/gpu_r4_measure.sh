#!/bin/bash
# round 4 validation, part 2: bench line, rocprofv3 kernel stats of the same command, PMC roofline evidence
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 420 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log > gpurun_out/bench_line.json
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/prof.log 2>&1 || exit 1
bash tools/gpu_pmc_r4.sh > gpurun_out/pmc_r4.log 2>&1
