"""Instruction mix of a kernel in a hipcc -S listing (offline ISA study).

usage: isa_mix.py file.s [kernel] -- counts by class over the kernel body, plus scratch ops."""
import re
import sys
from collections import Counter

path = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else None
body, on = [], False
for line in open(path):
    m = re.match(r"^([A-Za-z_][\w.]*):", line)
    if m and not m.group(1).startswith(".L"):
        on = want is None or m.group(1) == want
        continue
    if on and re.match(r"^\s+\.end_amdgpu_metadata|^\s+\.section", line):
        on = False
    if on:
        s = line.strip()
        if s and not s.startswith((".", ";", "//")) and not s.endswith(":"):
            body.append(s.split()[0])
c = Counter()
for op in body:
    p = op.split("_")
    cls = p[0] if p[0] in ("v", "s") else p[0]
    if p[0] == "v" and len(p) > 1:
        cls = "v_" + p[1]
    c[cls] += 1
print("total", len(body))
for k, v in c.most_common(40):
    print(f"{k:24s} {v}")
