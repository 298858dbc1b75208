cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gru_gpu.py tests/test_trained_gru_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gru.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/pytest_gru.log
for p in 0 1 0 1; do NPD_GRU_PIPE=$p timeout -k 10 120 python tools/gru_ab.py; done
