#!/usr/bin/env python3
"""Roofline numbers of the shipped GRU kernels from a PMC run of tools/pmc_gru_child.py (tools/gpu_pmc_r4.sh):

    python3 tools/pmc_gru_r4.py gpurun_out/pmc_gru > profiles/round4/pmc_gru_summary.json

Per kernel (counters averaged per launch by tools/pmc_summary.py; durations from the --kernel-trace --stats pass):
  * clock_ghz = GRBM_GUI_ACTIVE / 8 XCDs / kernel time (MI355X_MICROARCH.md 'DVFS give-back');
  * per_wave_step: MFMA busy cycles (SQ_VALU_MFMA_BUSY_CYCLES) and VALU active cycles (SQ_ACTIVE_INST_VALU, quad-cycles
    x 4) per wave and decoding step (waves = words / codewords per wave, 64 steps), and SQ_INSTS_VALU per wave-step;
  * simd_busy_frac = (MFMA busy + VALU active) / (1024 SIMDs x kernel cycles): ~1 means the two pipes' issue,
    serialised on a SIMD, fills the kernel;
  * mfma_frac_at_held_clock: MFMA busy / (1024 x kernel cycles) -- the fp32 kernel's bound, against the clock the
    chip held rather than the 2.4 GHz of the spec peak.
"""
import csv
import glob
import json
import os
import subprocess
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_gru"
WORDS, STEPS, SIMDS = 1 << 18, 64, 1024
CW_PER_WAVE = {"gru_decode_kernel": 32, "gru16p_kernel": 16}

summ = json.loads(subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "pmc_summary.py"), root],
                                 capture_output=True, text=True, check=True).stdout)
dur = {}
for f in glob.glob(os.path.join(root, "stats", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Name"].split("(")[0]] = float(r["AverageNs"])
out = {"source": "rocprofv3 --pmc (one pass) + --kernel-trace --stats over tools/pmc_gru_child.py: 2^18 Polar(64,32) "
                 "words at 2 dB, 3 launches per kernel", "kernels": {}}
for name, m in summ.items():
    short = next((k for k in CW_PER_WAVE if k in name), None)
    if short is None or name not in dur:
        continue
    t = dur[name] * 1e-9
    clock = m["GRBM_GUI_ACTIVE"] / 8 / t
    waves = WORDS / CW_PER_WAVE[short]
    ws = waves * STEPS
    mfma, valu = m["SQ_VALU_MFMA_BUSY_CYCLES"], 4 * m["SQ_ACTIVE_INST_VALU"]
    kcyc = SIMDS * clock * t
    out["kernels"][name] = dict(m, kernel_ms=t * 1e3, clock_ghz=clock / 1e9,
                                per_wave_step={"mfma_cycles": mfma / ws, "valu_cycles": valu / ws,
                                               "valu_insts": m["SQ_INSTS_VALU"] / ws},
                                simd_busy_frac=(mfma + valu) / kcyc, mfma_frac_at_held_clock=mfma / kcyc)
# flatten for bench.py's lookup by kernel name
for k, v in list(out["kernels"].items()):
    out[k] = v
print(json.dumps(out, indent=1))
