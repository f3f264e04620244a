#!/usr/bin/env python3
"""Instruction mix of the largest loop of a kernel in a .s file (static view:
VALU / LDS / SALU / VMEM / quarter-rate 32-bit multiplies per iteration).

    python tools/loopstats.py /tmp/wide.s k_wbitsILj2EjLb1E k_wpackILj2EjLb1ELi2E
"""
import re
import sys


def loop_stats(asm, pattern):
    starts = [m.start() for m in re.finditer(r'^(_Z\S*' + re.escape(pattern) + r'\S*):', asm, re.M)]
    out = []
    for i in starts:
        name = asm[i:asm.index(':', i)]
        j = asm.index('.Lfunc_end', i)
        lines = [l.strip() for l in asm[i:j].split('\n')]
        labels = {}
        for n, l in enumerate(lines):
            m = re.match(r'^(\.LBB\w+):', l)
            if m:
                labels[m.group(1)] = n
        best = None
        for n, l in enumerate(lines):
            m = re.match(r's_cbranch_\w+ (\.LBB\w+)|s_branch (\.LBB\w+)', l)
            if not m:
                continue
            t = m.group(1) or m.group(2)
            if t in labels and labels[t] < n:
                ins = [b for b in lines[labels[t]:n + 1] if b and not b.startswith(('.', ';'))]
                if best is None or len(ins) > best['len']:
                    best = {'len': len(ins),
                            'valu': sum(b.startswith('v_') for b in ins),
                            'lds': sum(b.startswith('ds_') for b in ins),
                            'salu': sum(b.startswith('s_') for b in ins),
                            'vmem': sum(b.startswith(('buffer_', 'global_', 'flat_')) for b in ins),
                            'mul32': sum(b.startswith(('v_mul_lo_u32', 'v_mul_hi_u32')) for b in ins)}
        out.append((name, best))
    return out


if __name__ == '__main__':
    asm = open(sys.argv[1]).read()
    for p in sys.argv[2:]:
        for name, st in loop_stats(asm, p):
            print(name, st)
