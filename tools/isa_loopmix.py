"""Instruction mix of the innermost-loop bodies of one kernel in a hipcc -S listing (by the compiler's
'Loop Header' comments): python tools/isa_loopmix.py build/asm/x.s <mangled-substring> [top-n]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
key = sys.argv[2]
i = s.index(key)
i = s.index(":", s.index("\n" + key[:0], i))
name_start = s.rfind("\n", 0, s.index(key + ":")) + 1
body = s[name_start:s.index(".Lfunc_end", name_start)].split("\n")
labels = {}
for n, l in enumerate(body):
    m = re.match(r"^(\.LBB\S+):", l.strip())
    if m:
        labels[m.group(1)] = n
best = None
for n, l in enumerate(body):
    m = re.match(r"^\s*s_cbranch_\w+\s+(\.LBB\S+)|^\s*s_branch\s+(\.LBB\S+)", l)
    if m:
        t = m.group(1) or m.group(2)
        if t in labels and labels[t] < n:
            span = (labels[t], n)
            if best is None or span[1] - span[0] > best[1] - best[0]:
                best = span
c = Counter()
for x in body[best[0]:best[1] + 1]:
    x = x.strip()
    if not x or x.startswith((".", ";")) or x.endswith(":"):
        continue
    op = x.split()[0]
    c[op[:2]] += 1
    c[op] += 1
print(f"largest loop lines {best}: VALU {c['v_']} SALU {c['s_']} DS {c['ds']} scratch {c['sc']}")
print(c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 30))
