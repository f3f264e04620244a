#!/usr/bin/env python3
"""Self-synchronisation distances of the workloads' Huffman codes (CPU, oracle
trees): for random bit offsets p, decode from p and record the bits until the
speculative path lands on a true codeword boundary. Sizes the warm-up window
of the single-pass index-free decoder."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import oracle as O  # noqa: E402


def stats(kind, n=1 << 21, samples=20000, seed=7):
    data = {"uniform": O.gen_uniform, "zipf": O.gen_zipf, "text": O.gen_text}[kind](0x5EED0001, n)
    tree = O.Tree.from_weights(O.weights_from_bytes(data))
    codes = tree.codes()
    lens = np.zeros(256, np.int64)
    for k, s in codes.items():
        lens[k] = len(s)
    bits = np.frombuffer("".join(codes[int(b)] for b in data).encode(), np.uint8) - 48
    B = bits.size
    bound = np.zeros(B + 1, bool)
    bound[np.concatenate([[0], np.cumsum(lens[data])])] = True
    trie = {}
    for k, s in codes.items():
        node = trie
        for ch in s[:-1]:
            node = node.setdefault(ch, {})
        node[s[-1]] = k
    rng = np.random.default_rng(seed)
    dist = []
    for p in rng.integers(0, B - 4096, samples):
        q = int(p)
        while not bound[q]:
            node = trie
            while True:
                node = node[chr(48 + bits[q])]
                q += 1
                if not isinstance(node, dict):
                    break
        dist.append(q - p)
    d = np.array(dist)
    mean = float(lens[data].mean())
    out = {"kind": kind, "mean_bits": round(mean, 3), "max_len": int(lens.max()),
           "p50": int(np.percentile(d, 50)), "p99": int(np.percentile(d, 99)), "max": int(d.max())}
    for w in (16, 32, 48, 64, 96, 128):
        out[f"P>{w}"] = float((d > w).mean())
    return out


if __name__ == "__main__":
    for k in sys.argv[1:] or ["zipf", "text", "uniform"]:
        print(stats(k), flush=True)
