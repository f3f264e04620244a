#!/usr/bin/env bash
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/enc_tests.log 2>&1
for ph in hist pack decode; do
  r=$(timeout -k 10 120 python tools/kbench.py --phase $ph --workload uniform --iters 20); echo "ph=$ph $r"
done > gpurun_out/enc_sweep.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/enc_bench.json 2>/dev/null
