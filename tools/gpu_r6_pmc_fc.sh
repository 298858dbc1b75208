#!/bin/bash
# Round-6 PMC of the final conv kernels (configs[4] fp16x3, tools/pmc_conv_child.py): HBM traffic (FETCH_SIZE /
# WRITE_SIZE, each in its own pass), TCC hit/miss, and the LDS / MFMA SQ group; then the same traffic pass with FC0's
# pre-split X (NPD_FC0_PRESPLIT=1), and a kernel-trace stats run.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/pmc_fc
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name env counters...
  local n=$1; shift; local e=$1; shift
  NPD_FC0_PRESPLIT=$e timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$n -o p -- \
      python3 tools/pmc_conv_child.py > $OUT/$n.log 2>&1
  local rc=$?; echo "pass $n ($*) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/$n.log; exit $rc; }
}
run p1 0 FETCH_SIZE
run p2 0 WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
run p3 0 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
run q1 1 FETCH_SIZE
NPD_FC0_PRESPLIT=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o s -- \
    python3 tools/pmc_conv_child.py > $OUT/stats.log 2>&1
echo "stats rc=$?"
