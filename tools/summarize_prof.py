#!/usr/bin/env python3
"""Summarise tools/profile.sh output: per kernel, average duration and the
per-dispatch averages of every collected counter (FETCH_SIZE doubled for
wide streaming reads per MI355X_MICROARCH.md §HBM is reported separately).

    python tools/summarize_prof.py gpurun_out/prof/<tag>
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    """the kernel's function name (k_hist1, k_decode_ring, ...), else a prefix"""
    m = re.search(r"\b(k_[A-Za-z0-9_]+)", name)
    if m:
        # the first template flag is LONG (codes > 32 bits) only for the pack
        # and the chunk decoder; elsewhere it is a layout or variant flag
        # (k_decode_fixed<PAD>: the swizzled stage) and the name stays plain
        long_flag = m.group(1) in ("k_pack", "k_decode") and ("<true" in name or "ILb1E" in name)
        return m.group(1) + ("<long>" if long_flag else "")
    return name[:40]


def main(d):
    res = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            res[short(r["Name"])]["avg_ms"] = float(r["AverageNs"]) / 1e6
            res[short(r["Name"])]["calls"] = int(r["Calls"])
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        acc = defaultdict(lambda: defaultdict(list))
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in acc.items():
            for c, vals in cs.items():
                # one row per dispatch and counter (values already summed over instances)
                res[k][c] = sum(vals) / max(1, len(vals))
    out = {}
    for k, v in res.items():
        if "FETCH_SIZE" in v:
            v["hbm_read_bytes_est"] = v["FETCH_SIZE"] * 1024 * 2  # KB units, x2 gfx950 wide-read correction
        if "WRITE_SIZE" in v:
            v["hbm_write_bytes_est"] = v["WRITE_SIZE"] * 1024
        out[k] = {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
