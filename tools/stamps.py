#!/usr/bin/env python3
"""Per-phase wave budgets from in-kernel s_memtime stamps (timing build).

    tools/build_variant.sh stamps "-DHUFF_STAMPS" csrc/device/indexless.hip \
        csrc/device/decode_wave.hip csrc/runtime/runtime.cpp
    HUFF_LIB_AB=stamps python tools/stamps.py --workload zipf

Runs the indexed decode and the index-free decode of a 1 GiB stream once
each (after warm-up calls), reads the stamp regions the timing build wrote
(runtime.cpp huff_diag_stamps; 10 words per wave, bitreader.hpp WaveStamps)
and prints one JSON line: per kernel, the mean / median cycles of every
phase of a wave, the wave lifetime, the kernel's span in cycles per
XCC (first entry to last stamp; s_memtime counters are per XCD) and the mean
number of waves resident per CU over it (sum of lifetimes / span / CUs).
s_memtime ticks at the shader clock.
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huff-encoding_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import huff_coding as H  # noqa: E402
from huff_coding import _lib  # noqa: E402
from huff_coding import device as D  # noqa: E402

SEEDS = {"uniform": 0x5EED0001, "zipf": 0x5EED0002, "text": 0x5EED0005}
PHASES = {
    "k_spec_lds": ["stage", "multi_walk", "exit_walk", "samples+barrier", "fixup"],
    "k_decode_fixed_skip": ["table", "input_stage", "skip_codes", "letters", "transpose", "stores"],
    "k_decode_fixed": ["table", "input_stage", "(skip)", "letters", "transpose", "stores"],
    "k_sync_decode": ["stage", "lead_in", "letters", "fixup", "look_back", "prefix", "out"],
}


def summarize(name, arr):
    """arr: (waves, 10) u64; stamps 0..7 (0 = not reached), [8] HW_ID, [9] XCC"""
    t = arr[:, :8].astype(np.int64)
    live = t[:, 0] > 0
    if not live.any():
        return {"waves": 0, "nonzero_words": int((arr != 0).sum()), "first_rows": arr[:3].tolist()}
    t = t[live]
    hw, xcc = arr[live, 8], arr[live, 9]
    nph = len(PHASES[name])
    res = {"waves": int(live.sum())}
    last = np.zeros(len(t), np.int64)
    for k in range(nph + 1):
        last = np.where(t[:, k] > 0, t[:, k], last)
    phases = {}
    prev = t[:, 0].copy()
    for k, ph in enumerate(PHASES[name], start=1):
        ok = t[:, k] > 0
        d = np.where(ok, t[:, k] - prev, 0)
        if ok.any():
            phases[ph] = {"mean": round(float(d[ok].mean()), 1), "median": float(np.median(d[ok])),
                          "p90": float(np.percentile(d[ok], 90)), "waves": int(ok.sum())}
        prev = np.where(ok, t[:, k], prev)
    life = last - t[:, 0]
    # s_memtime counters are per XCD (not synchronised): spans per XCC
    spans, resid = [], []
    for x in np.unique(xcc):
        m = xcc == x
        sp = int(last[m].max() - t[m, 0].min())
        ncu_x = len(np.unique((hw[m].astype(np.int64) >> 8) & 0xFF))
        spans.append(sp)
        resid.append(float(life[m].sum()) / max(sp, 1) / max(ncu_x, 1))
    cu = (xcc.astype(np.int64) << 16) | ((hw.astype(np.int64) >> 8) & 0xFF)
    ncu = len(np.unique(cu))
    res.update({"phases": phases, "lifetime": {"mean": round(float(life.mean()), 1),
                                               "median": float(np.median(life))},
                "span_cycles_per_xcc": {"mean": round(float(np.mean(spans)), 0), "max": int(max(spans))},
                "cus_seen": ncu, "resident_waves_per_cu": round(float(np.mean(resid)), 2)})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="zipf", choices=sorted(SEEDS))
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--seg", type=int, default=992, help="segment bits of the build (runtime.cpp HUFF_SEG_TARGET)")
    ap.add_argument("--walks", type=int, default=1, help="segments per thread of k_spec_lds")
    ap.add_argument("--sync", type=int, default=0,
                    help="segment bits of the one-pass decoder (syncdec.hip; HUFF_FIX_STATS prints them): "
                         "its stamps (region 0) instead of the pipeline's")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    L = C.CDLL(_lib.LIB_PATH)
    if not hasattr(L, "huff_diag_stamps"):
        sys.exit("not a timing build (HUFF_LIB_AB=stamps, built with -DHUFF_STAMPS)")
    L.huff_diag_stamps.argtypes = [C.c_int, C.c_void_p, C.c_size_t]
    ctx = H.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    n = args.bytes
    x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    D.generate(ctx, args.workload, SEEDS[args.workload], x.data_ptr(), n,
               cdf=D.zipf_cdf(1.2) if args.workload == "zipf" else None)
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    tree = H.HuffTree.from_weights(H.ByteWeights.from_array(job.hist()))
    bits = job.bits(tree)
    out = torch.empty((bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    job.pack(tree, out.data_ptr(), out.numel())
    comp_bytes, pad = (bits + 7) // 8, (8 - bits % 8) % 8
    for _ in range(3):
        job.decode(tree, out.data_ptr(), dec.data_ptr())
        D.decompress_dev(ctx, tree, out.data_ptr(), comp_bytes, pad, dec.data_ptr(), n + 64)
    torch.cuda.synchronize()
    assert torch.equal(dec[:n], x[:n])
    ntasks = (n + 4095) // 4096
    res = {"workload": args.workload, "n": n, "comp_bytes": comp_bytes}
    # the last index-free call left regions 0 and 1; the indexed decode region 2
    job.decode(tree, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    # segments of the speculative pass: runtime.cpp indexless_sync (args.seg bits for these trees)
    nseg = (bits + args.seg - 1) // args.seg
    per_wg = 256 * args.walks
    kernels = (("k_spec_lds", 0, (nseg + per_wg - 1) // per_wg * 4), ("k_decode_fixed_skip", 1, ntasks),
               ("k_decode_fixed", 2, ntasks))
    if args.sync:
        nseg = (bits + args.sync - 1) // args.sync
        kernels = (("k_sync_decode", 0, (nseg + 255) // 256 * 4), ("k_decode_fixed", 2, ntasks))
    for name, r, waves in kernels:
        buf = np.zeros((waves, 10), np.uint64)
        assert L.huff_diag_stamps(r, buf.ctypes.data, buf.size) == 0
        res[name] = summarize(name, buf)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
