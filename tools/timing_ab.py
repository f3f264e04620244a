#!/usr/bin/env python3
"""Does the per-phase HIP event timing (huff_ctx_set_timing) cost the bench
step time? The headline step (compress + decode of 1 GiB uniform, as
bench.py's run_workload) timed back to back with the library's kernel timing
on and off, alternated.

    python tools/timing_ab.py [--workload uniform] [--steps 20] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huff-encoding_amd"))

import torch  # noqa: E402

import huff_coding as H  # noqa: E402
from huff_coding import device as D  # noqa: E402

SEEDS = {"uniform": 0x5EED0001, "zipf": 0x5EED0002, "text": 0x5EED0005}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="uniform", choices=sorted(SEEDS))
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    ctx = H.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    n = args.bytes
    x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    D.generate(ctx, args.workload, SEEDS[args.workload], x.data_ptr(), n,
               cdf=D.zipf_cdf(1.2) if args.workload == "zipf" else None)
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    out = torch.empty(n + 128, dtype=torch.uint8, device="cuda")
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")

    def step():
        tree, bits = job.compress(out.data_ptr(), n + 128)
        job.decode(tree, out.data_ptr(), dec.data_ptr())

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    assert torch.equal(dec[:n], x[:n])
    res = {"workload": args.workload, "n": n, "steps": args.steps, "on": [], "off": []}
    for _ in range(args.reps):
        for mode in ("on", "off"):
            ctx.set_timing(mode == "on")
            ctx.reset_timing()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            res[mode].append(round((time.perf_counter() - t0) * 1e3 / args.steps, 4))
    ctx.set_timing(False)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
