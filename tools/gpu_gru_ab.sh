#!/bin/bash
# A/B of the F=64 split GRU kernels: NPD_GRU16=2 (pipelined) parity tests, then per-precision timing for each mode.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 0|1) return 0;; *) echo "stopping after rc=$1"; exit $1;; esac; }
NPD_GRU16=${MODE:-2} timeout -k 10 300 python -u -m pytest tests/test_gru_gpu.py tests/test_trained_gru_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gru_ab.log 2>&1
rc=$?; echo "gru pytest (mode ${MODE:-2}) rc=$rc"; tail -6 gpurun_out/pytest_gru_ab.log; stop $rc
for m in ${MODES:-1 2 1 2}; do
  NPD_GRU16=$m timeout -k 10 200 python -u tools/gru_prec.py > gpurun_out/gru_prec_$m.log 2>&1
  rc=$?; echo "mode $m rc=$rc"; grep -v amdgpu.ids gpurun_out/gru_prec_$m.log; stop $rc
done
exit 0
