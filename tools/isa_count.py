"""Instruction mix of one kernel in a hipcc -S listing: python tools/isa_count.py build/asm/x.s <mangled-substring>"""
import sys
from collections import Counter

s = open(sys.argv[1]).read()
key = sys.argv[2]
i = s.index(key + ":")
body = s[i:s.index(".Lfunc_end", i)].split("\n")
c = Counter()
for l in body:
    l = l.strip()
    if not l or l.startswith((".", ";")) or l.endswith(":"):
        continue
    op = l.split()[0]
    c[op[:2]] += 1
    c[op] += 1
print("VALU", c["v_"], "SALU", c["s_"], "LDS", c["ds"])
print(c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 25))
