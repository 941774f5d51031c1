#!/usr/bin/env python3
"""Per-kernel VGPR / scratch / LDS from hipcc -Rpass-analysis=kernel-resource-usage output (stdin)."""
import re
import sys

cur = None
rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
pat = sys.argv[1] if len(sys.argv) > 1 else ""
for k, v in rows.items():
    if pat in k:
        print(f"{v.get('VGPRs', '?'):>4} vgpr {v.get('AGPRs', '?'):>4} agpr {v.get('ScratchSize', '?'):>5} scr {v.get('LDS', '?'):>7} lds  {k}")
