#!/usr/bin/env python3
"""Join the host phase stamps of huff_enc_compress (HUFF_HOST_TRACE=1 lines,
steady_clock ns) with a rocprofv3 kernel trace of the same run (its
timestamps are on the host's monotonic clock): per step, how long the host
took to see pass 1's weights after k_hist_publish ended, the tree, the pass-2
launch call, and the launch call to the kernel's start.

    python tools/host_join.py host_trace.err trace/run_kernel_trace.csv
"""
import csv
import re
import statistics
import sys


def main():
    host = []
    for line in open(sys.argv[1]):
        m = re.search(r"at (\d+) (\d+) (\d+) (\d+) (\d+)", line)
        if m:
            host.append([int(v) for v in m.groups()])
    rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
    pub = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "k_hist_publish" in r["Kernel_Name"] or "k_rows_publish" in r["Kernel_Name"]]
    h1 = [int(r["Start_Timestamp"]) for r in rows if "k_hist1x2" in r["Kernel_Name"]]
    bm = [int(r["Start_Timestamp"]) for r in rows if "k_bytemap" in r["Kernel_Name"]]
    out = []
    for t0, t1, t2, tl, t3 in host:
        hs = [s for s in h1 if s >= t0 - 2000]
        if not hs:
            continue
        hstart = min(hs)
        pe = [e for s, e in pub if s >= hstart]
        ps = [s for s in bm if s >= t2]
        if not pe or not ps:
            continue
        pend, pstart = min(pe), min(ps)
        out.append(((hstart - t0) / 1e3, (t1 - pend) / 1e3, (t2 - t1) / 1e3, (tl - t2) / 1e3, (pstart - tl) / 1e3,
                    (pstart - pend) / 1e3))
    names = ("call->hist start", "publish end->host sees", "tree", "pack call", "launch->pack start", "idle total")
    print(f"{len(out)} steps joined")
    for i, n in enumerate(names):
        col = [o[i] for o in out]
        print(f"{n:24s} median {statistics.median(col):7.1f} us  min {min(col):7.1f}  max {max(col):7.1f}")


if __name__ == "__main__":
    main()
