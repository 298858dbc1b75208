#!/bin/bash
# round 5: one slice of the Polar(64,22) hidden-512 CRISP curriculum (run_crisp.sh's decoder) on the GPU.
#   PROBE=1: first time 40 steps of fp32 native GRU, MIOpen GRU and bf16 autocast (state in /tmp, nothing kept)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/train
C=trained_crisp_64_22_f512
if [ "${PROBE:-0}" = 1 ]; then
  for a in "" "--miopen" "--amp bf16" "--miopen --amp bf16"; do
    rm -f /tmp/probe.pt
    timeout -k 10 240 python -u tests/golden/train_crisp_gpu.py $C --state /tmp/probe.pt --out /tmp/probe.net.pt \
        --probe 40 $a 2>&1 | grep -E "PROBE|Error|error" | tee -a gpurun_out/train/probe.txt || exit 1
  done
fi
bash tools/gpu_train.sh ${BUDGET:-840} $C > gpurun_out/train/$C.txt 2>&1; echo "train rc=$?"
grep -E "eval|RESUME|DONE" gpurun_out/train/$C.txt | tail -n 12
