"""Static VALU/SALU/LDS instruction counts of one kernel in a -gline-tables-only .s file, per
source line (file:line of the innermost .loc), sorted by count; with --blocks, per basic block
with its line range.  Usage: isa_lines.py FILE.s KERNEL_SUBSTR [--blocks] [--lines a-b]"""
import re
import sys
from collections import Counter

path, ksub = sys.argv[1], sys.argv[2]
blocks = "--blocks" in sys.argv
txt = open(path).read().splitlines()
files = {}
start = end = None
for i, l in enumerate(txt):
    m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', l)
    if m:
        files[m.group(1)] = m.group(2)
    if start is None and re.match(r'^_Z\S*' + re.escape(ksub) + r'\S*:', l):
        start = i
    elif start is not None and l.startswith(".Lfunc_end"):
        end = i
        break
cur = "?"
cnt = Counter()
blk = []
bname = "entry"
bc = Counter()
blines = set()
for l in txt[start:end]:
    m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', l)
    if m:
        cur = f"{files.get(m.group(1), m.group(1)).split('/')[-1]}:{m.group(2)}"
        continue
    m = re.match(r'^(\.LBB\S+):', l)
    if m:
        blk.append((bname, dict(bc), sorted(blines)))
        bname, bc, blines = m.group(1), Counter(), set()
        continue
    s = l.strip()
    if not s or s.startswith((".", ";")):
        continue
    op = s.split()[0]
    k = "v" if op.startswith("v_") else "s" if op.startswith("s_") else "ds" if op.startswith("ds_") else "mem" if op.startswith(("buffer_", "global_", "flat_")) else "o"
    cnt[(cur, k)] += 1
    bc[k] += 1
    blines.add(cur)
blk.append((bname, dict(bc), sorted(blines)))
if blocks:
    for b, c, ls in blk:
        print(f"{b:16s} v={c.get('v',0):4d} s={c.get('s',0):4d} ds={c.get('ds',0):3d} mem={c.get('mem',0):3d}  {' '.join(ls[:8])}")
else:
    tot = Counter()
    for (ln, k), n in cnt.items():
        tot[k] += n
    print("total", dict(tot))
    for (ln, k), n in sorted(cnt.items(), key=lambda x: -x[1])[:80]:
        if k == "v":
            print(f"{n:5d} {k} {ln}")
