#!/usr/bin/env python3
"""Summarise rocprofv3 SQLite outputs (run_results.db): per kernel, the
average dispatch duration (kernel-trace runs) and the per-dispatch average of
every PMC counter (--pmc runs).

    python tools/rocpd_summary.py out.json "<what>" dir1 [dir2 ...]
"""
import glob
import json
import os
import re
import sqlite3
import sys
from collections import defaultdict


def short(n):
    m = re.search(r"\b(k_[A-Za-z0-9_]+)", n or "")
    return m.group(1) if m else (n or "")[:40]


def main(out, what, dirs):
    res = defaultdict(dict)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
            c = sqlite3.connect(f)
            views = {r[0] for r in c.execute("select name from sqlite_master")}
            if "counters_collection" in views:
                cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
                acc = defaultdict(lambda: defaultdict(list))
                for r in c.execute("select * from counters_collection"):
                    x = dict(zip(cols, r))
                    acc[short(x["kernel_name"])][x["counter_name"]].append(x["value"])
                for k, cs in acc.items():
                    for cn, v in cs.items():
                        res[k][cn] = sum(v) / len(v)
            if "kernels" in views:
                cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
                dur = defaultdict(list)
                for r in c.execute("select * from kernels"):
                    x = dict(zip(cols, r))
                    dur[short(x["name"])].append((x["end"] - x["start"]) / 1e6)
                for k, v in dur.items():
                    if v and "avg_ms" not in res[k]:
                        res[k]["avg_ms"] = sum(v) / len(v)
                        res[k]["dispatches"] = len(v)
    for k, x in res.items():
        if x.get("SQ_LDS_IDX_ACTIVE"):
            x["lds_conflict_frac"] = x.get("SQ_LDS_BANK_CONFLICT", 0) / x["SQ_LDS_IDX_ACTIVE"]
        if "FETCH_SIZE" in x:
            x["fetch_bytes_x2"] = x["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in x:
            x["write_bytes"] = x["WRITE_SIZE"] * 1024
    doc = {"what": what, "kernels": {k: {kk: round(vv, 4) for kk, vv in x.items()} for k, x in sorted(res.items())}}
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
