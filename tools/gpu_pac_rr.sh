cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
NPD_LIB=tools/bin/libnpd_rr.so timeout -k 10 300 python -u -m pytest tests/test_sc_gpu.py -q -x -k "pac or PAC" --timeout 200 --timeout-method thread > gpurun_out/pytest_rr.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_rr.log
[ $rc -eq 0 ] || exit $rc
echo "== cur" && timeout -k 10 200 python -u tools/pac_bench.py && \
echo "== rr" && NPD_LIB=tools/bin/libnpd_rr.so timeout -k 10 200 python -u tools/pac_bench.py && \
echo "== cur" && timeout -k 10 200 python -u tools/pac_bench.py
