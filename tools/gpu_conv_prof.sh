#!/bin/bash
# per-kernel conv forward times under rocprofv3 (--kernel-trace --stats) for each library given (NPD_LIB), configs[4]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/conv_prof
i=0
for lib in "$@"; do
  i=$((i + 1))
  NPD_LIB=$(readlink -f $lib) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/conv_prof/p$i -o run -- \
    python3 tools/conv_time.py 1 > gpurun_out/conv_prof/p$i.log 2>&1 || { echo "prof $lib failed"; tail -20 gpurun_out/conv_prof/p$i.log; exit 1; }
  f=$(find gpurun_out/conv_prof/p$i -name "*kernel_stats.csv" | head -1)
  echo "== $lib"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows:
    n=r['Name']
    if 'conv' in n or 'fc_' in n or 'layernorm' in n:
        print(f\"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us  {n[:110]}\")
"
done
