cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for pf in 1 0 1 0; do echo "NPD_SC_PF=$pf"; NPD_SC_PF=$pf timeout -k 10 120 python tools/pac_bench.py; done
timeout -k 10 400 python -u -m pytest tests/test_sc_gpu.py -q -x --timeout 200 --timeout-method thread -k "not anchors" > gpurun_out/pytest_sc.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_sc.log
