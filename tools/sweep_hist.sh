#!/usr/bin/env bash
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "weights or medium or threaded or stitching" > gpurun_out/hist_tests.log 2>&1
for w in uniform zipf; do
  r=$(timeout -k 10 120 python tools/kbench.py --phase hist --workload $w --iters 20); echo "w=$w $r"
done > gpurun_out/hist_sweep.log 2>&1
