#!/usr/bin/env python3
"""Debug helper for the single-pass index-free decoder: decode oracle-written
streams through huff_dev_decompress with HUFF_IFD=1 and =0 and report where
the outputs differ (or where bytes past the letters were written)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "huff-encoding_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import huff_coding as H  # noqa: E402
import oracle as O  # noqa: E402
from huff_coding import device as D  # noqa: E402


def run(name, data, ctx):
    t = O.Tree.from_weights(O.weights_from_bytes(data))
    code, ln = t.code_table()
    host = np.frombuffer(data, np.uint8)
    comp, bits = O.fast_encode(host, code, ln, threads=8)
    pad = (8 - bits % 8) % 8
    tree = H.HuffTree.try_from_bin(t.as_bin())
    dc = torch.zeros(comp.size + 64, dtype=torch.uint8, device="cuda")
    dc[: comp.size] = torch.from_numpy(comp).cuda()
    n = len(data)
    for flag in ("1", "0"):
        os.environ["HUFF_IFD"] = flag
        out = torch.full((n + 80,), 0xAB, dtype=torch.uint8, device="cuda")
        got = D.decompress_dev(ctx, tree, dc.data_ptr(), comp.size, pad, out.data_ptr(), n + 16)
        torch.cuda.synchronize()
        res = out.cpu().numpy()
        bad = np.nonzero(res[:n] != host)[0]
        past = np.nonzero(res[n:] != 0xAB)[0]
        print(f"{name} ifd={flag} n={n} got={got} bits={bits} pad={pad} wrong={bad.size} first={bad[:5].tolist()} "
              f"past={past.size} {res[n:n + past.size].tolist() if past.size else ''}", flush=True)


def main():
    ctx = H.Context(0)
    os.environ["HUFF_IFD_TRACE"] = "1"
    rng = np.random.default_rng(2024)
    run("uniform40", rng.integers(0, 40, 3_000_001, dtype=np.uint8).tobytes(), ctx)
    for n in (1000, 65537, 100_001, 1_000_003):
        run(f"u40-{n}", rng.integers(0, 40, n, dtype=np.uint8).tobytes(), ctx)


main()
