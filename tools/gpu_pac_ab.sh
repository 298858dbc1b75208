cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sc_gpu.py tests/test_empty_gpu.py tests/test_eval_loops_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_pac.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_pac.log
[ $rc -eq 0 ] || exit $rc
for m in 0; do
NPD_SC_ROOT=$m timeout -k 10 300 python -u -m pytest tests/test_sc_gpu.py -q -x -k "pac or PAC" --timeout 200 --timeout-method thread > gpurun_out/pytest_root$m.log 2>&1; rc=$?; echo "pytest root$m rc=$rc"; tail -2 gpurun_out/pytest_root$m.log
[ $rc -eq 0 ] || exit $rc
done
for m in 1 0 1 0; do
  echo "== NPD_SC_ROOT=$m"; NPD_SC_ROOT=$m timeout -k 10 200 python -u tools/pac_bench.py || exit 1
done
echo "== base"; NPD_LIB=tools/bin/libnpd_base.so timeout -k 10 200 python -u tools/pac_bench.py
