cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gru_gpu.py tests/test_trained_gru_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gru16.log 2>&1; echo "pytest rc=$?"; tail -15 gpurun_out/pytest_gru16.log
timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --no-conv --no-scl --no-lse --no-mc --no-pac > gpurun_out/bench_gru16.log 2>&1; echo "bench rc=$?"
python - <<'PY'
import json
l=[x for x in open('gpurun_out/bench_gru16.log') if x.startswith('{')][-1]
d=json.loads(l); g=d['crisp_gru']
for k in ('fp16x3','bf16x3','bf16'): print(k, {a:b for a,b in g[k].items() if a!='note'})
print('fp32', g['avg_launch_ms'], g['frac'])
PY
