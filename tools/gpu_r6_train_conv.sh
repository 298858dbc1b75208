#!/bin/bash
# round 6: one slice of the embed-128 conv curriculum (tests/golden/train_conv_gpu.py, run_alt.sh's configuration with
# shortened stages).  The resumable state travels in train_r6/ (copy gpurun_out/train/conv_e128.pt there after a call).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/train
[ -f train_r6/conv_e128.pt ] && cp train_r6/conv_e128.pt gpurun_out/train/conv_e128.pt
if [ -n "$PROBE" ]; then
  for a in "" "--native" "--amp bf16" "--native --amp bf16"; do
    rm -f /tmp/probe.pt
    timeout -k 10 300 python -u tests/golden/train_conv_gpu.py --state /tmp/probe.pt --out /tmp/probe_w.pt --probe $PROBE $a \
      2>&1 | grep -E "PROBE|Error" | sed "s/^/[$a] /"
  done
  exit 0
fi
timeout -k 10 $((${BUDGET:-960} + 200)) python -u tests/golden/train_conv_gpu.py --state gpurun_out/train/conv_e128.pt \
    --out gpurun_out/train/conv_e128.net.pt --budget-s ${BUDGET:-960} ${TRAIN_ARGS:-} > gpurun_out/train/conv_e128.txt 2>&1
echo "train rc=$?"
grep -E "eval|RESUME|DONE|Error|stage .* step (600|1200|24000)/" gpurun_out/train/conv_e128.txt | tail -n 30
