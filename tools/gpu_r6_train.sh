#!/bin/bash
# round 6: one slice of a GPU curriculum from tests/golden/crisp_cases.py (CASE, default configs[2]'s decoder on the full
# run_crisp.sh schedule, trained_crisp_64_32_full), HIP-graph replayed training steps.  The resumable state travels
# in train_r6/ (uploaded with the tree; copy gpurun_out/train/$C.pt there after each call).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/train
C=${CASE:-trained_crisp_64_32_full}
[ -f train_r6/$C.pt ] && cp train_r6/$C.pt gpurun_out/train/$C.pt
timeout -k 10 $((${BUDGET:-960} + 150)) python -u tests/golden/train_crisp_gpu.py $C --state gpurun_out/train/$C.pt \
    --out gpurun_out/train/$C.net.pt --budget-s ${BUDGET:-960} --graph --eval-every 5000 > gpurun_out/train/$C.txt 2>&1
echo "train rc=$?"
grep -E "eval|RESUME|DONE|Error" gpurun_out/train/$C.txt | tail -n 12
