#!/usr/bin/env python3
"""Diagnose the checked decoder builds (HUFF_DEC_VARIANT 11-13) on one GPU:
for each case, decode, catch the self-check error, and locate the wrong
letters by task / workgroup / lane / letter index."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huff-encoding_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import huff_coding as H  # noqa: E402
from huff_coding import device as D  # noqa: E402


def run(ctx, kind, n, var, grid=None, reps=2):
    os.environ["HUFF_DEC_VARIANT"] = var
    os.environ["HUFF_DISABLE_FIXED8"] = "1"
    if grid:
        os.environ["HUFF_DEC_GRID"] = str(grid)
    else:
        os.environ.pop("HUFF_DEC_GRID", None)
    if kind == "geo":  # codes longer than the 12-bit table (the SLOW body)
        rng = np.random.default_rng(77)
        host = np.minimum(rng.geometric(0.45, n) - 1, 255).astype(np.uint8)
        host[rng.integers(0, n, 3000)] = rng.integers(0, 256, 3000, dtype=np.uint8)
        x = torch.from_numpy(np.concatenate([host, np.zeros(64, np.uint8)])).cuda()
    else:
        seed = {"uniform": 0x5EED0001, "zipf": 0x5EED0002, "text": 0x5EED0005}[kind]
        x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        D.generate(ctx, kind, seed, x.data_ptr(), n, cdf=D.zipf_cdf(1.2) if kind == "zipf" else None)
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    tree = H.HuffTree.from_weights(H.ByteWeights.from_array(job.hist()))
    bits = job.bits(tree)
    out = torch.zeros((bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
    job.pack(tree, out.data_ptr(), out.numel())
    res = []
    for _ in range(reps):
        dec = torch.zeros(n + 64, dtype=torch.uint8, device="cuda")
        err = None
        try:
            job.decode(tree, out.data_ptr(), dec.data_ptr())
        except H.HuffError as e:
            err = str(e)
        torch.cuda.synchronize()
        bad = (dec[:n] != x[:n]).cpu().numpy()
        idx = np.nonzero(bad)[0]
        lanes = np.unique(idx // 64)
        tasks = np.unique(idx // 4096)
        first_in_lane = {}
        for li in lanes[:6]:
            first_in_lane[int(li)] = int(idx[idx // 64 == li][0] % 64)
        dumps = []
        if lanes.size:
            xs = x[:n].cpu().numpy()
            ds = dec[:n].cpu().numpy()
            _, ln = tree.code_table()
            cl = ln[xs].astype(np.int64)
            cum = np.concatenate([[0], np.cumsum(cl)])
            for li in lanes[:3]:
                s0 = int(li) * 64
                dumps.append({"lane": int(li), "start_bit": int(cum[s0]),
                              "want": xs[s0:s0 + 64].tolist(), "got": ds[s0:s0 + 64].tolist(),
                              "len": cl[s0:s0 + 64].tolist()})
        res.append({"err": err, "bad_bytes": int(idx.size), "bad_lanes": int(lanes.size),
                    "bad_tasks": [int(t) for t in tasks[:12]], "ntasks_bad": int(tasks.size),
                    "first_letter_in_lane": first_in_lane, "dumps": dumps,
                    "lane_in_task": sorted(set(int(l % 64) for l in lanes[:200]))[:20]})
    return {"kind": kind, "n": n, "var": var, "grid": grid, "runs": res}


def main():
    torch.cuda.set_device(0)
    ctx = H.Context(0)
    out = []
    M = 1 << 20
    cases = [("geo", 16 * M, "14", None), ("geo", 64 * M, "14", None)]
    if len(sys.argv) > 1:  # kind:n:variant ... (n in MiB)
        cases = [(c.split(":")[0], int(c.split(":")[1]) * M, c.split(":")[2],
                  int(c.split(":")[3]) if len(c.split(":")) > 3 else None) for c in sys.argv[1:]]
    for kind, n, var, grid in cases:
        r = run(ctx, kind, n, var, grid)
        print(json.dumps(r), flush=True)
        out.append(r)


if __name__ == "__main__":
    main()
