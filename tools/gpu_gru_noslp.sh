#!/bin/bash
# A/B: npd_gru.hip built with -fno-slp-vectorize (tools/bin/libnpd_noslp.so) against the default build -- GRU parity
# tests on the variant, then alternating timings of the four precision paths
cd "$GRAFT_REPO_ROOT" || exit 1
NPD_LIB=tools/bin/libnpd_noslp.so timeout -k 10 300 python -u -m pytest tests/test_gru_gpu.py tests/test_trained_gru_gpu.py tests/test_gru_precision_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gru_noslp.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/pytest_gru_noslp.log
for v in base noslp base noslp; do
  if [ $v = noslp ]; then export NPD_LIB=tools/bin/libnpd_noslp.so; else unset NPD_LIB; fi
  echo "== $v"; timeout -k 10 200 python -u tools/gru_prec.py || exit 1
done
