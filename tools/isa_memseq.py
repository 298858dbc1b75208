"""Compressed sequence of memory / wait / scratch instructions of one kernel in a hipcc -S listing:
python tools/isa_memseq.py build/asm/x.s <mangled-substring>"""
import sys

s = open(sys.argv[1]).read()
key = sys.argv[2]
i = s.index(key)
i = s.rfind("\n", 0, s.index(":", i)) + 1
j = s.index(".Lfunc_end", i)
body = s[i:j].split("\n")
prev = None
cnt = 0
first = 0
prevt = ""
for n, l in enumerate(body):
    t = l.strip()
    if not t.startswith(("global_", "s_waitcnt", "ds_", "flat_", "buffer_", "scratch_", "s_cbranch", "s_branch")) and not (t.startswith(".LBB") and t.endswith(":")):
        continue
    k = t.split()[0]
    if k == prev:
        cnt += 1
        continue
    if prev:
        print(f"{first:5d} {prevt}" + (f"  x{cnt}" if cnt > 1 else ""))
    prev, prevt, cnt, first = k, t.split(";")[0][:70], 1, n
print(f"{first:5d} {prevt}" + (f"  x{cnt}" if cnt > 1 else ""))
