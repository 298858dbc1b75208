#!/usr/bin/env python3
"""Per-dispatch-shape PMC summary: rocprofv3 --pmc CSVs grouped by (kernel, grid size), so launches of one
kernel with different shapes (e.g. the conv layers' 64- and 128-channel grids) are told apart.
python tools/pmc_dispatch.py gpurun_out/pmc [kernel-substring]"""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
flt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if flt not in k:
            continue
        key = f"{k} grid={r.get('Grid_Size', '?')} lds={r.get('LDS_Block_Size', r.get('Lds_Block_Size', '?'))}"
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, d in agg.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    m["launches"] = max(len(v) for v in d.values())
    wc = m.get("SQ_WAVE_CYCLES") or m.get("SQ_BUSY_CYCLES")
    if wc:
        for c in list(m):
            if c.startswith("SQ_") and c not in ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES") and "CYCLES" in c or c.startswith("SQ_WAIT") or c.startswith("SQ_ACTIVE"):
                m[c + "_per_wave_cycle"] = m[c] / m["SQ_WAVE_CYCLES"] if "SQ_WAVE_CYCLES" in m else None
    if "SQ_BUSY_CYCLES" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m and m["SQ_BUSY_CYCLES"]:
        m["mfma_busy_frac_of_sq_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / m["SQ_BUSY_CYCLES"]
    out[k] = m
print(json.dumps(out, indent=1))
