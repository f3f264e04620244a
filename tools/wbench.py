#!/usr/bin/env python3
"""Wider-letter path timings (include/huffgpu_wide.h) on HBM-resident input.

    python tools/wbench.py --width 2 --mb 1024 --iters 10

Letters: `--width` bytes each, 1 GiB by default, drawn on the device from a
Zipf(1.1)-like law over a random alphabet of `--alphabet` letters. Prints one
JSON line: per-kernel average ms (HIP events around each launch) and GB/s of
input letters, plus the algorithmic HBM bytes of each kernel.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huff-encoding_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import huff_coding as H  # noqa: E402
import huff_coding.wide as W  # noqa: E402

TORCH = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}
NP = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=2, choices=[1, 2, 4, 8])
    ap.add_argument("--mb", type=int, default=1024)
    ap.add_argument("--alphabet", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--indexless", action="store_true")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    ctx = H.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    Wd = args.width
    n = (args.mb << 20) // Wd
    g = torch.Generator(device="cuda").manual_seed(7)
    k = min(args.alphabet, 1 << (8 * Wd)) if Wd < 8 else args.alphabet
    rng = np.random.default_rng(7)
    if Wd == 1:
        alpha = np.arange(256, dtype=np.uint8)[:k]
    else:
        alpha = np.unique(rng.integers(0, np.iinfo(NP[Wd]).max, 4 * k, dtype=NP[Wd], endpoint=True))[:k]
    rng.shuffle(alpha)
    p = 1.0 / np.arange(1, alpha.size + 1) ** 1.1
    p /= p.sum()
    idx = torch.multinomial(torch.tensor(p, device="cuda", dtype=torch.float32), n, replacement=True, generator=g)
    a_dev = torch.from_numpy(alpha.view(np.int64 if Wd == 8 else {1: np.uint8, 2: np.int16, 4: np.int32}[Wd])).cuda()
    x = a_dev[idx].contiguous()
    del idx
    assert x.data_ptr() % 16 == 0
    letters_host = None
    # weights map (timed once; a sort of n letters)
    ctx.set_timing(True)
    ctx.reset_timing()
    letters_host = x.cpu().numpy().view(NP[Wd])
    wmap = W.build_weights_map(letters_host, ctx)  # host-buffer API: includes the H2D copy
    wm_ms, _ = ctx.kernel_time("wweights")
    t = W.WideTree.from_weights(list(wmap.items()), NP[Wd])
    job = W.WideEncodeJob(ctx, Wd, x.data_ptr(), n)
    bits = job.bits(t)
    out = torch.empty((bits + 31) // 32 * 4 + 16, dtype=torch.uint8, device="cuda")
    dec = torch.empty_like(x)
    job.pack(t, out.data_ptr(), out.numel())
    job.decode(t, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dec, x), "round trip"
    ctx.reset_timing()
    for _ in range(args.iters):
        job.bits(t)
        job.pack(t, out.data_ptr(), out.numel())
        job.decode(t, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    comp = (bits + 7) // 8
    nbytes = n * Wd
    res = {"width": Wd, "letters": n, "input_bytes": nbytes, "alphabet": int(alpha.size),
           "bits_per_letter": round(bits / n, 4), "weights_map_ms": round(wm_ms, 3), "kernels": {}}
    algo = {"wbits": nbytes, "wscan": 0, "wpack": nbytes + comp, "wdecode": comp + nbytes}
    for kname, b in algo.items():
        ms, c = ctx.kernel_time(kname)
        if c:
            avg = ms / c
            gbps = b / (avg * 1e-3) / 1e9 if b else None
            res["kernels"][kname] = {"avg_ms": round(avg, 4), "algo_bytes": b,
                                     "GBps": round(gbps, 1) if b else None,
                                     "frac_of_8TBps": round(gbps / 8000, 4) if b else None}
    enc_ms = sum(res["kernels"][k]["avg_ms"] for k in ("wbits", "wscan", "wpack"))
    res["encode_GBps_input"] = round(nbytes / (enc_ms * 1e-3) / 1e9, 1)
    res["encode_frac_input"] = round(nbytes / (enc_ms * 1e-3) / 1e9 / 8000, 4)
    res["decode_GBps_input"] = round(nbytes / (res["kernels"]["wdecode"]["avg_ms"] * 1e-3) / 1e9, 1)
    if args.indexless:
        pad = (8 - bits % 8) % 8
        ctx.reset_timing()
        times = []
        for _ in range(3):  # the first call builds the shape's tables and workspaces
            dec.zero_()
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            cnt = W.decompress_dev(ctx, t, out.data_ptr(), comp, pad, dec.data_ptr(), n)
            ev1.record()
            torch.cuda.synchronize()
            assert cnt == n and torch.equal(dec, x)
            times.append(ev0.elapsed_time(ev1))
        res["indexless_decode_ms_cold"] = round(times[0], 3)
        res["indexless_decode_ms"] = round(min(times[1:]), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
