#!/usr/bin/env python3
"""Per-kernel resource summary of a gfx950 assembly listing (hipcc -S --cuda-device-only):
VGPRs, LDS bytes, scratch, VALU / LDS / global-memory instruction counts, s_set_gpr_idx.
usage: isa_stats.py listing.s [substring ...]   (kernels whose mangled name holds every substring)"""
import re
import sys

s = open(sys.argv[1]).read()
want = sys.argv[2:]
for m in re.finditer(r"^(_Z\w+):", s, re.M):
    n = m.group(1)
    if not all(w in n for w in want) or ".amdhsa_kernel " + n not in s:
        continue
    body = s[m.start():s.index(".Lfunc_end", m.start())]
    lines = [l.strip() for l in body.split("\n")]
    meta = s[s.index(".amdhsa_kernel " + n):][:4000]
    get = lambda k: re.search(r"\.amdhsa_%s (\d+)" % k, meta).group(1)
    cnt = lambda p: sum(1 for l in lines if re.match(p, l))
    print(f"{n[:90]:90s} vgpr {get('next_free_vgpr'):>4} lds {get('group_segment_fixed_size'):>6} "
          f"scratch {get('private_segment_fixed_size')} valu {cnt(r'v_')} ds {cnt(r'ds_')} "
          f"vmem {cnt(r'(global|buffer)_(load|store)')} gidx {body.count('s_set_gpr_idx_on')}")
