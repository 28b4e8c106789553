"""Instruction mix of one kernel in a hipcc -S listing: python tools/isa_mix.py <file.s> <substr>"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
key = sys.argv[2]
m = re.search(r"^(\S*%s\S*):\s*;" % re.escape(key), s, re.M)
start = m.end()
end = s.index(".Lfunc_end", start)
body = s[start:end]
ins = []
for line in body.split("\n"):
    t = line.strip()
    if not t or t.startswith((".", ";")) or t.endswith(":"):
        continue
    ins.append(t.split()[0])
c = collections.Counter(ins)
print(m.group(1))
print("total", len(ins), "valu", sum(v for k, v in c.items() if k.startswith("v_")),
      "salu", sum(v for k, v in c.items() if k.startswith("s_")),
      "ds", sum(v for k, v in c.items() if k.startswith("ds_")),
      "vmem", sum(v for k, v in c.items() if k.startswith(("global_", "buffer_"))))
for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
    print(f"{v:6d} {k}")
