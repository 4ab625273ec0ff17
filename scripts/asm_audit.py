"""Audit of an asm-owned-accumulator kernel in a gfx950 assembly listing: compiler-placed accumulator
traffic outside the inline-asm statements, scratch use, highest arch VGPR, instruction mix per loop block.
    python scripts/asm_audit.py file.s MANGLED_NAME"""
import re
import sys
from collections import Counter

text = open(sys.argv[1]).read()
name = sys.argv[2]
body = re.search(rf"^{name}:(.*?)^\.Lfunc_end", text, re.S | re.M).group(1)
inasm, bad, vmax = False, [], 0
for line in body.splitlines():
    if ";;#ASMSTART" in line:
        inasm = True
        continue
    if ";;#ASMEND" in line:
        inasm = False
        continue
    code = line.split(";")[0]
    for m in re.finditer(r"\bv\[?(\d+)(?::(\d+))?", code):
        vmax = max(vmax, int(m.group(2) or m.group(1)))
    if not inasm and re.search(r"v_accvgpr|[\s,]a\[?\d", code):
        bad.append(line.strip())
print("compiler accumulator traffic:", len(bad), bad[:6])
print("scratch:", "scratch_" in body, " max arch vgpr:", vmax)
blocks, cur = [], None
for l in body.splitlines():
    if re.match(r"^\.LBB\d+_\d+:", l) or re.match(r"^; %bb", l):
        cur = [l.strip()[:40], []]
        blocks.append(cur)
        continue
    s = l.split(";")[0].strip()
    if s and not s.startswith(".") and cur:
        cur[1].append(s)
for b in blocks:
    if len(b[1]) < 40:
        continue
    c = Counter()
    for i in b[1]:
        op = i.split()[0]
        k = ("mfma" if "mfma" in op else "ds_read" if op.startswith("ds_read") else "buffer" if op.startswith("buffer")
             else "waitcnt" if "waitcnt" in op else "s_nop" if op == "s_nop" else "accvgpr" if "accvgpr" in op
             else "salu" if op.startswith("s_") else "valu" if op.startswith("v_") else op)
        c[k] += 1
    print(b[0], len(b[1]), dict(c.most_common()))
