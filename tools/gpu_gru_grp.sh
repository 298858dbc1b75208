cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gru_gpu.py tests/test_trained_gru_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_grp.log 2>&1 && echo "pytest ok" && tail -2 gpurun_out/pytest_grp.log && \
echo "== grouped" && timeout -k 10 200 python -u tools/gru_prec.py && \
echo "== plain" && NPD_GRU_GROUPED=0 timeout -k 10 200 python -u tools/gru_prec.py
