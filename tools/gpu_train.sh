#!/bin/bash
# One gpurun slice of the GPU curriculum stages (tests/golden/train_crisp_gpu.py), resumable:
#   tools/gpu_train.sh BUDGET_S CASE [CASE ...]
# train_state/CASE.pt (copied back from gpurun_out/train/ after each call) carries the state between calls.
set -e
B=$1; shift
mkdir -p gpurun_out/train
for c in "$@"; do
  [ -f train_state/$c.pt ] && cp train_state/$c.pt gpurun_out/train/$c.pt
  INIT=""
  [ -f train_state/$c.init.pt ] && INIT="--init train_state/$c.init.pt"
  timeout -k 10 $((B + 120)) python -u tests/golden/train_crisp_gpu.py $c --state gpurun_out/train/$c.pt \
      --out gpurun_out/train/$c.net.pt --budget-s $B $INIT ${TRAIN_ARGS:-} 2>&1 | tee -a gpurun_out/train/$c.log
done
