#!/usr/bin/env python3
"""CPU analysis of tools/diag_src.py output (profiles/r02/n_early_loads/
diag_src.jsonl): rebuild the same uniform stream with the oracle, and for each
failing lane find which stream dword ORed at which lane bit turns the right
window bits into the decoded ones (got == want | dword d at bit o)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


def main(path):
    n = 1 << 24
    x = O.gen_uniform(0x5EED0001, n)
    t = O.Tree.from_weights(O.weights_from_array(O.fast_hist(x, 8)))
    code, ln = t.code_table()
    assert (ln == 8).all()
    code = code.astype(np.uint8)
    stream = code[x]  # every code is 8 bits: stream byte j = code of letter j
    lanes = {}
    for line in open(path):
        for e in json.loads(line)["examples_not_found"]:
            lanes.setdefault(e["pos"] - e["pos"] % 64, []).append(e)
    bits = lambda b: np.unpackbits(np.asarray(b, np.uint8)).astype(int)  # noqa: E731
    for ls, es in lanes.items():
        want = stream[ls:ls + 64].copy()
        got = want.copy()
        for e in es:
            g, p = int(e["got"], 16), e["pos"] - ls
            for i in range(4):
                got[p + i] = code[(g >> (8 * i)) & 255]
        wb, gb = bits(want), bits(got)
        fits = []
        t0 = ls - ls % 4096
        for d in range(t0 // 4 - 64, t0 // 4 + 1088):
            wd = bits(stream[4 * d:4 * d + 4])
            for o in range(200, 330):
                P = np.zeros(512, int)
                hi = min(o + 32, 512)
                P[o:hi] = wd[:hi - o]
                if ((wb | P) == gb).all():
                    fits.append((d - ls // 4, o))
        print(json.dumps({"lane_start_byte": ls, "task": ls // 4096, "lane": (ls % 4096) // 64,
                          "extra_bits": np.nonzero(gb & ~wb)[0].tolist(), "lost_bits": np.nonzero(wb & ~gb)[0].tolist(),
                          "fits_dword_at_bit": fits[:6]}))


main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles/r02/n_early_loads/diag_src.jsonl"))
