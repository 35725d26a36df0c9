#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in the saved gfx950 assembly.
    python tools/isa_blocks.py <kernel-name-substring> [min_instructions]"""
import re
import sys
from collections import Counter

S = sys.argv[3] if len(sys.argv) > 3 else "enet-csharp_amd/build/crc32_kernels-hip-amdgcn-amd-amdhsa-gfx950.s"
pat = sys.argv[1]
mn = int(sys.argv[2]) if len(sys.argv) > 2 else 20
lines = open(S).read().split("\n")
i = next(k for k, l in enumerate(lines) if re.match(r"^_Z\w+:", l) and pat in l)
end = next(j for j in range(i, len(lines)) if lines[j].strip().startswith("s_endpgm"))
body = [l.strip() for l in lines[i:end]]
blocks, cur, cnt = [], "entry", Counter()
for l in body[1:]:
    if l.startswith(".LBB") or l.startswith("; %bb."):
        blocks.append((cur, cnt))
        cur, cnt = l[:48], Counter()
        continue
    if not l or l.startswith((";", ".")):
        continue
    op = l.split()[0]
    t = "ds" if op.startswith("ds_") else "glds" if "load_lds" in op else "v" if op.startswith("v_") else "s" if op.startswith("s_") else op
    cnt[t] += 1
    if op in ("v_perm_b32",):
        cnt["perm"] += 1
blocks.append((cur, cnt))
for name, c in blocks:
    if sum(v for k, v in c.items() if k != "perm") >= mn:
        print(f"{name:50s} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
