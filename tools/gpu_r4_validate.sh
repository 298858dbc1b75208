#!/bin/bash
# round 4 validation, part 1: the full GPU test suite and smoke(), then the GRU precision study on the trained
# Polar(64,32) fixture (profiles/round4/gru_precision.json)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 780 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/gru_precision.py --n 65536 --out gpurun_out/gru_precision.json > gpurun_out/gru_precision.log 2>&1
