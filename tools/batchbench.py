#!/usr/bin/env python3
"""Batched small-stream trees (huff_batch_hist / huff_batch_trees) on
HBM-resident streams: kernel times of both launches, streams per second, and
the library's own host build of the same trees (huff_tree_from_weights +
as_bin, one thread) beside them.

    python tools/batchbench.py --streams 10000 --bytes 16384 --iters 10
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huff-encoding_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import huff_coding as H  # noqa: E402
from huff_coding import batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=10000)
    ap.add_argument("--bytes", type=int, default=16384, help="bytes per stream")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cpu-sample", type=int, default=500, help="streams built on the host for comparison")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    ctx = H.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    S, L = args.streams, args.bytes
    g = torch.Generator(device="cuda").manual_seed(5)
    # skewed bytes, a different skew per stream: floor(256 u^k), k in [1.5, 6)
    u = torch.rand((S, L), device="cuda", generator=g)
    k = 1.5 + 4.5 * torch.rand((S, 1), device="cuda", generator=g)
    data = torch.clamp(torch.floor(256 * u ** k), 0, 255).to(torch.uint8)
    data = data.reshape(-1).contiguous()
    offs = torch.arange(0, S + 1, device="cuda", dtype=torch.int64) * L
    hist = batch.batch_hist(ctx, data, offs)
    t = batch.batch_trees(ctx, hist)
    torch.cuda.synchronize()
    ctx.set_timing(True)
    ctx.reset_timing()
    for _ in range(args.iters):
        batch.batch_hist(ctx, data, offs)
        batch.batch_trees(ctx, hist)
    torch.cuda.synchronize()
    res = {"streams": S, "bytes_per_stream": L, "iters": args.iters}
    for k in ("hist_batch", "tree_batch"):
        ms, c = ctx.kernel_time(k)
        res[k + "_ms"] = round(ms / c, 4)
    res["trees_per_s"] = round(S / (res["tree_batch_ms"] * 1e-3))
    res["hist_GBps"] = round(S * L / (res["hist_batch_ms"] * 1e-3) / 1e9, 1)
    # the host build of the same trees (one thread, through the C ABI)
    h = hist[: args.cpu_sample].cpu().numpy()
    ws = [H.ByteWeights.from_array(r) for r in h]
    t0 = time.perf_counter()
    for w in ws:
        H.HuffTree.from_weights(w).as_bin()
    el = time.perf_counter() - t0
    res["host_trees_per_s"] = round(len(ws) / el)
    res["host_note"] = "huff_tree_from_weights + huff_tree_as_bin per stream (host/tree.cpp), 1 thread, Python loop"
    st = t.status.cpu().numpy()
    res["status_counts"] = {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
