#!/bin/bash
# round 4 close-out.  PART=tests: the full pytest -m gpu suite and smoke(); PART=bench: the bench line and the
# rocprofv3 --kernel-trace --stats summary of the same command (the bench runs its own FETCH_SIZE / WRITE_SIZE passes)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${PART:-tests}" = tests ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/pytest_gpu.log | tail -n 8
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1; echo "smoke rc=$?"
  tail -n 2 gpurun_out/smoke.txt
else
  timeout -k 10 500 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -n 20 gpurun_out/bench.log; exit 1; }
  tail -n 1 gpurun_out/bench.log > gpurun_out/bench_line.json
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py \
      --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/prof.log 2>&1; echo "rocprof rc=$?"
  python3 -c "
import json; d = json.load(open('gpurun_out/bench_line.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'])
for k in ('metric_as_named', 'pac_sc', 'conv_model', 'crisp_gru', 'pac_gru'):
    v = d.get(k) or {}
    print(k, v.get('value'), (v.get('roofline') or {}).get('frac') if isinstance(v.get('roofline'), dict) else v.get('frac'))
"
fi
