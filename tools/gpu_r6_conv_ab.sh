#!/bin/bash
# A/B of an environment switch over the configs[4] conv forward: per-kernel times under rocprofv3 --kernel-trace --stats
#   AB_VAR=NPD_FC0_PRESPLIT bash tools/gpu_r6_conv_ab.sh 0 1 [0 1 ...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=${AB_OUT:-gpurun_out/conv_ab}
mkdir -p $OUT
i=0
for v in "$@"; do
  i=$((i + 1))
  env $AB_VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$i -o run -- \
    python3 tools/conv_time.py 2 > $OUT/p$i.log 2>&1 || { echo "prof $AB_VAR=$v failed"; tail -20 $OUT/p$i.log; exit 1; }
  f=$(find $OUT/p$i -name "*kernel_stats.csv" | head -1)
  echo "== $AB_VAR=$v"; grep "ms per" $OUT/p$i.log; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if 'conv' in n or 'fc_' in n or 'layernorm' in n or 'split' in n:
        print(f\"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us  {n[:110]}\")
"
done
