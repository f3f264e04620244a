#!/usr/bin/env python3
"""Where do the reproducer's wrong letters come from? Uniform 16 MiB input
(every code 8 bits, so stream byte j encodes letter j): decode with the
library selected by HUFF_LIB_AB, and for every wrong dword of a lane (4
letters) find where in the input the 4 letters it decoded actually sit
(4-byte aligned positions), relative to where they should come from."""
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huff-encoding_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import huff_coding as H  # noqa: E402
from huff_coding import device as D  # noqa: E402


def main():
    ctx = H.Context(0)
    n = 1 << 24
    os.environ["HUFF_DISABLE_FIXED8"] = "1"
    x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    D.generate(ctx, "uniform", 0x5EED0001, x.data_ptr(), n)
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    tree = H.HuffTree.from_weights(H.ByteWeights.from_array(job.hist()))
    bits = job.bits(tree)
    assert bits == 8 * n
    out = torch.zeros(n + 64, dtype=torch.uint8, device="cuda")
    job.pack(tree, out.data_ptr(), out.numel())
    ref = x[:n].cpu().numpy()
    words = ref.view(np.uint32)
    where = collections.defaultdict(list)
    for i, w in enumerate(words.tolist()):
        where[w].append(4 * i)
    for rep in range(3):
        dec = torch.zeros(n + 64, dtype=torch.uint8, device="cuda")
        job.decode(tree, out.data_ptr(), dec.data_ptr())
        torch.cuda.synchronize()
        got = dec[:n].cpu().numpy()
        gw = got.view(np.uint32)
        bad = np.nonzero(gw != words)[0]
        deltas = collections.Counter()
        kinds = collections.Counter()
        examples = []
        for i in bad.tolist():
            w = int(gw[i])
            pos = 4 * i
            cand = where.get(w, [])
            if w == 0:
                kinds["zero"] += 1
            if not cand:
                kinds["not_in_input"] += 1
                if len(examples) < 6:
                    examples.append({"pos": pos, "got": hex(w), "want": hex(int(words[i]))})
                continue
            d = min(cand, key=lambda p: abs(p - pos)) - pos
            deltas[d] += 1
            kinds["found"] += 1
        tasks = np.unique(bad * 4 // 4096)
        print(json.dumps({"rep": rep, "wrong_dwords": int(bad.size), "wrong_tasks": int(tasks.size),
                          "lane_dword_hist": collections.Counter(((bad * 4) % 64 // 4).tolist()).most_common(8),
                          "kinds": dict(kinds), "top_deltas_bytes": deltas.most_common(12),
                          "examples_not_found": examples}), flush=True)


main()
