#!/usr/bin/env python3
"""Turn a tools/summarize_prof.py summary into profiles/traffic_<workload>.json:
per kernel, HBM bytes per launch from the PMC passes (FETCH_SIZE x 1024 x 2:
the gfx950 wide-streaming-read correction of MI355X_MICROARCH.md; WRITE_SIZE
x 1024). bench.py reports the dominant kernel's figure as roofline.traffic.

    python tools/make_traffic.py gpurun_out/r01/prof_all_uniform.json uniform
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(src, workload):
    d = json.load(open(src))
    out = {"_source": os.path.relpath(src, ROOT) if os.path.isabs(src) else src,
           "_note": "per-launch averages; read = FETCH_SIZE*1024*2 (exact for 16-B streaming reads, "
                    "uncalibrated for other access shapes), write = WRITE_SIZE*1024"}
    for k, v in d.items():
        if not k.startswith("k_") or "FETCH_SIZE" not in v or "WRITE_SIZE" not in v:
            continue
        r = v["FETCH_SIZE"] * 1024 * 2
        w = v["WRITE_SIZE"] * 1024
        out[k] = {"hbm_read_bytes": round(r), "hbm_write_bytes": round(w), "hbm_bytes": round(r + w),
                  "avg_ms": v.get("avg_ms")}
    dst = os.path.join(ROOT, "profiles", f"traffic_{workload}.json")
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    print(dst)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
