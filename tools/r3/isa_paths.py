"""VALU instructions per basic block of one kernel in a hipcc -S listing, and the count along
each path through its wave-uniform branches (tools/r3: the executed VALU per wave of a kernel
with s_cbranch_scc branches is not its static count).
    python tools/r3/isa_paths.py <file.s> <symbol-substring>"""
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r"^(\S*%s\S*):\s*;" % re.escape(sys.argv[2]), s, re.M)
body = s[m.end():s.index(".Lfunc_end", m.end())]
blocks, cur, name = [], [], "entry"
for line in body.split("\n"):
    t = line.strip()
    if re.match(r"^\.LBB\S+:", t):
        blocks.append((name, cur)); name, cur = t[:-1].split()[0].rstrip(":"), []
        continue
    if not t or t.startswith((".", ";")):
        continue
    cur.append(t.split()[0] if not t.startswith("s_cbranch") and not t.startswith("s_branch") else t)
blocks.append((name, cur))
for nm, ins in blocks:
    v = sum(1 for i in ins if i.startswith("v_"))
    br = [i for i in ins if i.startswith(("s_cbranch", "s_branch"))]
    print(f"{nm:12s} valu {v:5d}  {' | '.join(br)}")
