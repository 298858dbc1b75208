cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sc_gpu.py tests/test_empty_gpu.py tests/test_eval_loops_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_pac.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_pac.log
[ $rc -eq 0 ] || exit $rc
for v in rr r2; do
NPD_LIB=tools/bin/libnpd_$v.so timeout -k 10 300 python -u -m pytest tests/test_sc_gpu.py -q -x -k "pac or PAC" --timeout 200 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1; rc=$?; echo "pytest $v rc=$rc"; tail -2 gpurun_out/pytest_$v.log
[ $rc -eq 0 ] || exit $rc
done
for lib in "" tools/bin/libnpd_rr.so tools/bin/libnpd_r2.so tools/bin/libnpd_base.so ""; do
  echo "== ${lib:-cur}"; NPD_LIB=${lib:-neural_polar_decoder_amd/libnpd.so} timeout -k 10 200 python -u tools/pac_bench.py || exit 1
done
