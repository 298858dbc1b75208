#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc/p*/p_counter_collection.csv) per kernel.

HBM traffic per launch follows MI355X_MICROARCH.md 'HBM': FETCH_SIZE reads 1/2 of the bytes of a wide
coalesced streaming read on gfx950 (doubled here); WRITE_SIZE is exact for 16-B/lane streaming stores.
Both are in KiB.
"""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, d in agg.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        m["hbm_bytes_per_launch_corrected"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
    if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
        for c in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY"):
            if c in m:
                m[c + "_frac"] = m[c] / m["SQ_WAVE_CYCLES"]
    out[k] = m
print(json.dumps(out, indent=1))
