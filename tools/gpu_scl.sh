cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_scl_gpu.py tests/test_eval_loops_gpu.py tests/test_sc_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_scl.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/pytest_scl.log
timeout -k 10 120 python tools/scl_bench.py
timeout -k 10 120 python tools/pac_bench.py
