#!/bin/bash
# A/B of folding the gate exp2 constants into the GRU weights (VAR=NPD_GRU_FOLD: the fp16x3 split of the 16-codeword
# kernels, unscaled + folded vs x 2^8 scaled; VAR=NPD_GRU_FOLD32: the fp32 F <= 64 kernel), after the GRU parity
# tests on the default.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 0|1) return 0;; *) echo "stopping after rc=$1"; exit $1;; esac; }
env ${TESTENV:-NPD_X=0} timeout -k 10 300 python -u -m pytest tests/test_gru_gpu.py tests/test_trained_gru_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gru_fold.log 2>&1
rc=$?; echo "gru pytest rc=$rc"; tail -15 gpurun_out/pytest_gru_fold.log; stop $rc
VAR=${VAR:-NPD_GRU_FOLD}
for f in 1 0 1 0; do
  env $VAR=$f timeout -k 10 200 python -u tools/gru_prec.py > gpurun_out/gru_prec_${VAR}$f.log 2>&1
  rc=$?; echo "$VAR=$f rc=$rc"; grep -v amdgpu.ids gpurun_out/gru_prec_${VAR}$f.log | head -2; stop $rc
done
exit 0
