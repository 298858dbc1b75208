cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sc_gpu.py tests/test_empty_gpu.py tests/test_eval_loops_gpu.py tests/test_trained_gru_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_pac.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_pac.log
[ $rc -eq 0 ] || exit $rc
echo "== new" && timeout -k 10 200 python -u tools/pac_bench.py && \
echo "== base" && NPD_LIB=tools/bin/libnpd_base.so timeout -k 10 200 python -u tools/pac_bench.py && \
echo "== new" && timeout -k 10 200 python -u tools/pac_bench.py
