#!/usr/bin/env python3
"""Idle gaps inside the headline step from a rocprofv3 kernel trace
(`--kernel-trace --output-format csv`): per block of back-to-back steps (a
block ends at an idle gap above --split us), the median duration of each
step kernel and of the idle time before it.

    python tools/step_gaps.py gpurun_out/x/trace/run_kernel_trace.csv
"""
import argparse
import csv
import statistics


def short(name):
    for k in ("k_hist1x2", "k_rows_sum", "k_rows_publish", "k_hist_publish", "k_bytemap", "k_pack", "k_decode", "k_chunk_bits",
              "k_scan"):
        if k in name:
            return k
    return name[:24] or "copy"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--split", type=float, default=2000.0)
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "calib" not in r["Kernel_Name"] and "at::native" not in r["Kernel_Name"]]
    blocks, cur, prev_end, last = [], [], None, ""
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if prev_end is not None and (s - prev_end) / 1e3 > args.split and cur:
            blocks.append(cur)
            cur = []
        gap = 0.0 if prev_end is None or not cur else max(0.0, (s - prev_end) / 1e3)
        name = short(r["Kernel_Name"])
        if name == "k_bytemap":  # serial steps: pass 2 follows pass 1, decode follows pass 2
            name = "k_bytemap(after pass 1)" if last in ("k_hist_publish", "k_rows_sum", "k_rows_publish") else "k_bytemap(after bytemap)"
        if not name.startswith("__amd"):
            last = name
        cur.append((name, (e - s) / 1e3, gap))
        prev_end = e if prev_end is None else max(prev_end, e)
    if cur:
        blocks.append(cur)
    for i, b in enumerate(blocks):
        if len(b) < 10:
            continue
        span = {}
        for name, dur, gap in b[1:]:
            span.setdefault(name, ([], []))
            span[name][0].append(dur)
            span[name][1].append(gap)
        parts = [f"{k} {statistics.median(d):.1f} (+{statistics.median(g):.1f} idle)" for k, (d, g) in span.items()]
        print(f"block {i}: {len(b)} kernels; " + "; ".join(parts))


if __name__ == "__main__":
    main()
