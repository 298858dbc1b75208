cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gru_gpu.py tests/test_trained_gru_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gru16.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gru16.log
timeout -k 10 200 python -u tools/gru_prec.py
