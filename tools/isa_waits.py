#!/usr/bin/env python3
"""Summarise s_waitcnt / LDS-DMA / ds_read counts per staged-kernel variant in the
saved gfx950 assembly (make isa)."""
import re, sys
from collections import Counter
S = sys.argv[1] if len(sys.argv) > 1 else "enet-csharp_amd/build/crc32_kernels-hip-amdgcn-amd-amdhsa-gfx950.s"
pat = sys.argv[2] if len(sys.argv) > 2 else "staged_kernel"
lines = open(S).read().split("\n")
for i, l in enumerate(lines):
    m = re.match(r"^(_Z\w+):\s", l)
    if not m or pat not in m.group(1):
        continue
    end = next(j for j in range(i, len(lines)) if lines[j].strip().startswith("s_endpgm"))
    body = [x.strip() for x in lines[i:end]]
    c = Counter(x.split(";")[0].strip() for x in body if x.startswith("s_waitcnt"))
    print(m.group(1), f"{end - i} lines  glds={sum('global_load_lds' in x for x in body)}"
          f"  ds_read={sum(x.startswith('ds_read') for x in body)}  readlane={sum('readlane' in x for x in body)}")
    for k, v in c.most_common(10):
        print(f"   {v:4d} {k}")
