cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; echo "bench rc=$?"
python - <<'PY'
import json
l=[x for x in open('gpurun_out/bench.log') if x.startswith('{')][-1]
d=json.loads(l)
print({k: d[k] for k in ('value','ms_per_step','ber_match','ber_db_offset')})
m=d.get('metric_as_named',{}); print('MAN', m.get('value'), m.get('roofline',{}).get('frac'), m.get('fp16x3_path',{}).get('value'), m.get('gru_vs_reference'), m.get('cpu_baseline',{}).get('value'))
print('MCPAC', d.get('montecarlo_pac'))
print('PACSC', d.get('pac_sc',{}).get('avg_launch_ms'), d.get('pac_sc',{}).get('roofline'))
print('SCL', d.get('scl',{}).get('polar_256_128_L4'))
print('LSE', d.get('sc_lse'))
PY
