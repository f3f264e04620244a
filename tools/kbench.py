#!/usr/bin/env python3
"""Kernel microbenchmark for profiling: repeat one phase of the hot path.

    python tools/kbench.py --phase pack --workload zipf --iters 20

phase: hist | pack | decode | all. Inputs are generated on the device once;
the selected phase is launched `iters` times back to back so rocprofv3
(--kernel-trace / --pmc) sees many identical dispatches.
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
from huff_coding import device as D  # noqa: E402

SEEDS = {"uniform": 0x5EED0001, "zipf": 0x5EED0002, "text": 0x5EED0005}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--phase", default="all", choices=["hist", "pack", "decode", "indexless", "all"])
    ap.add_argument("--workload", default="uniform", choices=sorted(SEEDS))
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-verify", action="store_true", help="timing experiments on builds that skip work")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    ctx = H.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    n = args.bytes
    x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    D.generate(ctx, args.workload, SEEDS[args.workload], x.data_ptr(), n,
               cdf=D.zipf_cdf(1.2) if args.workload == "zipf" else None)
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    w = job.hist()
    if args.phase == "hist":  # timing of pass 1 alone (also for experiment builds)
        ctx.set_timing(True)
        ctx.reset_timing()
        for _ in range(args.iters):
            job.hist()
        torch.cuda.synchronize()
        ms, c = ctx.kernel_time("hist")
        print(json.dumps({"phase": "hist", "workload": args.workload, "n": n, "iters": args.iters, "hist_ms": ms / c}))
        return
    tree = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
    bits = job.bits(tree)
    out = torch.empty((bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    job.pack(tree, out.data_ptr(), out.numel())
    job.decode(tree, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    if not args.no_verify:
        assert torch.equal(dec[:n], x[:n])
    if args.phase == "indexless":  # decode without the restart index (reference-written streams)
        comp_bytes = (bits + 7) // 8
        pad = (8 - bits % 8) % 8
        got = D.decompress_dev(ctx, tree, out.data_ptr(), comp_bytes, pad, dec.data_ptr(), n + 64)
        torch.cuda.synchronize()
        assert args.no_verify or (got == n and torch.equal(dec[:n], x[:n]))
        ctx.set_timing(True)
        ctx.reset_timing()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            D.decompress_dev(ctx, tree, out.data_ptr(), comp_bytes, pad, dec.data_ptr(), n + 64)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) * 1e3 / args.iters
        res = {"phase": "indexless", "workload": args.workload, "n": n, "comp_bytes": comp_bytes,
               "wall_ms_per_iter": el, "GBps_out": n / el / 1e6}
        ms, c = ctx.kernel_time("indexless_decode")
        if c:
            res["ifd_kernel_ms"] = ms / c
        print(json.dumps(res))
        return
    ctx.set_timing(True)
    ctx.reset_timing()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        if args.phase in ("hist", "all"):
            job.hist()
        if args.phase in ("pack", "all"):
            job.pack(tree, out.data_ptr(), out.numel())
        if args.phase in ("decode", "all"):
            job.decode(tree, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    res = {"phase": args.phase, "workload": args.workload, "n": n, "comp_bytes": (bits + 7) // 8,
           "iters": args.iters, "wall_ms_per_iter": el * 1e3 / args.iters}
    for k in ("hist", "chunk_bits", "scan", "pack", "decode"):
        ms, c = ctx.kernel_time(k)
        if c:
            res[k + "_ms"] = ms / c
    print(json.dumps(res))


if __name__ == "__main__":
    main()
