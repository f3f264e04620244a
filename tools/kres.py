#!/usr/bin/env python3
"""Per-kernel VGPRs / scratch / occupancy from -Rpass-analysis=kernel-resource-usage
remarks on stdin (or a .res file): python tools/kres.py [regex] < remarks"""
import re
import sys

pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        cur = {'name': m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, rx in (('vgpr', r'VGPRs: (\d+)'), ('scratch', r'ScratchSize \[bytes/lane\]: (\d+)'),
                    ('occ', r'Occupancy \[waves/SIMD\]: (\d+)'), ('lds', r'LDS Size \[bytes/block\]: (\d+)')):
        m = re.search(rx, line)
        if m:
            cur[key] = int(m.group(1))
for r in rows:
    if pat and not pat.search(r['name']):
        continue
    n = re.sub(r'^_ZN4huff3dev12_GLOBAL__N_1\d+', '', r['name'])
    print(f"{n:60s} vgpr={r.get('vgpr')} scratch={r.get('scratch')} occ={r.get('occ')} lds={r.get('lds')}")
