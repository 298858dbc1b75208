#!/bin/bash
# round 4: finish the Polar(32,16) K = 16 GPU stage, then continue the F = 512 PAC(128,64) curriculum
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_train.sh 300 trained_crisp_32_16 > gpurun_out/train_32_16.txt 2>&1; echo "train32 rc=$?"
tail -n 3 gpurun_out/train_32_16.txt
B=${F512_BUDGET:-840}
bash tools/gpu_train.sh $B trained_pac_128_64_f512 > gpurun_out/train_f512.txt 2>&1; echo "trainf512 rc=$?"
grep -E "eval|RESUME|DONE" gpurun_out/train_f512.txt | tail -n 8
