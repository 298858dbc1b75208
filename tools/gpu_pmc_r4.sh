#!/bin/bash
# round 4 roofline evidence: PMC of the shipped GRU kernels (fp32 gru_decode_kernel<64,2>, fp16x3
# gru16p_kernel<5>) and HBM traffic of the streaming PAC(128,64) SC kernel.
set -e
PMC_CHILD=tools/pmc_gru_child.py PMC_OUT=gpurun_out/pmc_gru bash tools/gpu_pmc_k.sh \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
PMC_CHILD=tools/pmc_pac.py PMC_OUT=gpurun_out/pmc_pac bash tools/gpu_pmc_k.sh FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
python3 tools/pmc_summary.py gpurun_out/pmc_gru > gpurun_out/pmc_gru/summary.json
python3 tools/pmc_summary.py gpurun_out/pmc_pac > gpurun_out/pmc_pac/summary.json
python3 tools/pmc_gru_r4.py gpurun_out/pmc_gru > gpurun_out/pmc_gru/pmc_gru_summary.json
