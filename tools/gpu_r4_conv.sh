#!/bin/bash
# round 4: conv fp16x3 kernels (weight-stationary conv layers, 128 x 128 FC tile) -- parity tests, timing, rocprof --
# then a slice of the F = 512 PAC curriculum (F512_BUDGET seconds, 0 = none)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_trained_conv_gpu.py -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 25 gpurun_out/pytest_conv.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/conv_time.py 2 > gpurun_out/conv_time.txt 2>&1 || exit 1
cat gpurun_out/conv_time.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_conv -o conv -- \
    python3 tools/conv_time.py 1 > gpurun_out/prof_conv.log 2>&1 || exit 1
f=$(find gpurun_out/prof_conv -name "*kernel_stats.csv" | head -n 1); cut -c1-150 "$f" | head -n 14
timeout -k 10 400 python -u tools/conv_precision.py --out gpurun_out/conv_precision.json > gpurun_out/conv_precision.log 2>&1
echo "convprec rc=$?"; tail -n 3 gpurun_out/conv_precision.log | cut -c1-400
B=${F512_BUDGET:-0}
if [ "$B" -gt 0 ]; then
  bash tools/gpu_train.sh $B trained_pac_128_64_f512 > gpurun_out/train_f512.txt 2>&1; echo "trainf512 rc=$?"
  grep -E "eval|RESUME|DONE" gpurun_out/train_f512.txt | tail -n 8
fi
