"""Instruction mix of each loop (backward branch target .. branch) of one kernel in a hipcc -S listing:
python tools/isa_loop.py build/asm/x.s <mangled-name> [top-n]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
key = sys.argv[2]
i = s.index(key + ":")
body = [l.strip() for l in s[i:s.index(".Lfunc_end", i)].split("\n")]
labels = {l[:-1]: n for n, l in enumerate(body) if re.match(r"^\.LBB\S+:$", l)}
for n, l in enumerate(body):
    m = re.match(r"^s_cbranch_\w+\s+(\.LBB\S+)|^s_branch\s+(\.LBB\S+)", l)
    if not m:
        continue
    tgt = m.group(1) or m.group(2)
    if tgt in labels and labels[tgt] < n:
        c = Counter()
        for x in body[labels[tgt]:n + 1]:
            if not x or x.startswith((".", ";")) or x.endswith(":"):
                continue
            op = x.split()[0]
            c[op[:2]] += 1
            c[op] += 1
        print(f"loop {tgt} lines {labels[tgt]}..{n}: VALU {c['v_']} SALU {c['s_']} LDS {c['ds']}")
        print("  ", c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 30))
