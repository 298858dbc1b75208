"""Per-kernel register / scratch / lane-spill summary of a hipcc -S listing:
python tools/kres.py build/asm/x.s [substring]"""
import re
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", s, re.S):
    name, body = m.group(1), m.group(2)
    if flt not in name:
        continue
    vg = int(re.search(r"next_free_vgpr (\d+)", body).group(1))
    sc = int(re.search(r"private_segment_fixed_size (\d+)", body).group(1))
    lds = re.search(r"group_segment_fixed_size (\d+)", body)
    i = s.find(name + ":")
    j = s.find(".Lfunc_end", i)
    text = s[i:j]
    wl, rl = text.count("v_writelane"), text.count("v_readlane")
    print(f"{vg:4d} vgpr  {sc:5d} B scratch  writelane {wl:4d} readlane {rl:4d}  {name[:110]}")
