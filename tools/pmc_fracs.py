"""Per-kernel issue / LDS / wait fractions from a PMC directory (tools/gpu_pmc_k.sh) and the kernel-trace stats
of the same program: python tools/pmc_fracs.py gpurun_out/pmck > profiles/roundN/pmc_secondary.json

  clock_ghz        GRBM_GUI_ACTIVE / 8 XCDs / average kernel time (MI355X_MICROARCH.md 'DVFS give-back')
  valu_issue_frac  SQ_INSTS_VALU (wave-instructions) / time / 1.2288e12 (1024 SIMDs x 2.4 GHz x one wave64
                   VALU instruction per 2 cycles, the SIMD-32 issue rate with >= 2 waves)
  lds_array_frac   SQ_LDS_IDX_ACTIVE / 256 CUs / kernel cycles (LDS-array busy cycles per CU)
  *_frac of waves  SQ_WAIT_ANY, SQ_ACTIVE_INST_VALU, SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
"""
import csv
import glob
import json
import subprocess
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmck"
summ = json.loads(subprocess.run([sys.executable, "tools/pmc_summary.py", root], capture_output=True, text=True).stdout)
dur = {}
for f in glob.glob(f"{root}/stats/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Name"].split("(")[0]] = float(r["AverageNs"]) * 1e-9
out = {}
for k, m in summ.items():
    if "npd::" not in k or k not in dur:
        continue
    t = dur[k]
    cyc = m.get("GRBM_GUI_ACTIVE", 0.0) / 8
    o = {"avg_us": t * 1e6, "clock_ghz": cyc / t / 1e9 if t else None,
         "valu_wave_instr": m.get("SQ_INSTS_VALU"), "valu_issue_frac": m.get("SQ_INSTS_VALU", 0.0) / t / 1.2288e12,
         "lds_wave_instr": m.get("SQ_INSTS_LDS"),
         "lds_array_frac": m.get("SQ_LDS_IDX_ACTIVE", 0.0) / 256 / cyc if cyc else None,
         "lds_bank_conflict_cycles": m.get("SQ_LDS_BANK_CONFLICT")}
    for c in ("SQ_WAIT_ANY_frac", "SQ_ACTIVE_INST_VALU_frac", "SQ_WAIT_INST_ANY_frac"):
        if c in m:
            o[c.replace("SQ_", "").lower()] = m[c]
    out[k.replace("void ", "")] = o
print(json.dumps(out, indent=1))
