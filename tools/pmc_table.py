#!/usr/bin/env python3
"""Per-kernel resource table from rocprofv3 csv dirs (kernel trace + PMC
passes): duration, VALU and LDS busy fractions (VALU: wave64 instructions x 2
cycles per SIMD; LDS: SQ_LDS_IDX_ACTIVE per CU), bank-conflict share, HBM
bytes (FETCH_SIZE doubled for 16-B streaming reads, MI355X_MICROARCH.md).

    python tools/pmc_table.py gpurun_out/r3u indexless [out.json]
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

CUS, SIMDS, CLK = 256, 1024, 2.4e9


def short(n):
    m = re.search(r"\b(k_[A-Za-z0-9_]+)", n)
    return m.group(1) if m else n[:30]


def table(d, prefix):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/{prefix}_*/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = defaultdict(list)
    for f in glob.glob(f"{d}/{prefix}_trace/*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = {}
    for k, cs in acc.items():
        if not k.startswith("k_") or k.startswith("k_gen"):
            continue
        ms = sum(dur[k]) / len(dur[k]) if dur.get(k) else 0.0
        c = {n: sum(v) / len(v) for n, v in cs.items()}
        cyc = ms * 1e-3 * CLK
        row = {"avg_ms": round(ms, 4)}
        if cyc:
            row["valu_busy"] = round(c.get("SQ_INSTS_VALU", 0) / SIMDS * 2 / cyc, 3)
            row["lds_busy"] = round(c.get("SQ_LDS_IDX_ACTIVE", 0) / CUS / cyc, 3)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            row["lds_conflict_share"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 3)
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                  "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES"):
            if n in c:
                row[n] = round(c[n])
        if "FETCH_SIZE" in c:
            row["hbm_read_bytes"] = round(c["FETCH_SIZE"] * 1024 * 2)
        if "WRITE_SIZE" in c:
            row["hbm_write_bytes"] = round(c["WRITE_SIZE"] * 1024)
        out[k] = row
    return out


if __name__ == "__main__":
    t = table(sys.argv[1], sys.argv[2])
    for k, r in t.items():
        print(f"{k:24s} {r.get('avg_ms', 0):.3f} ms  VALU {r.get('valu_busy', 0):.2f}  LDS {r.get('lds_busy', 0):.2f}"
              f" (conflicts {r.get('lds_conflict_share', 0):.2f})  rd {r.get('hbm_read_bytes', 0) / 1e9:.3f} GB"
              f"  wr {r.get('hbm_write_bytes', 0) / 1e9:.3f} GB")
    if len(sys.argv) > 3:
        json.dump(t, open(sys.argv[3], "w"), indent=1)
