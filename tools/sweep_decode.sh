#!/usr/bin/env bash
# decode kernel variants (HUFF_DEC_VARIANT) on the three workloads + parity
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "medium or long or foreign or stitching or full_size_zipf" > gpurun_out/dec_tests.log 2>&1
for w in zipf text uniform; do for v in 0 1 2; do
  r=$(HUFF_DISABLE_FIXED8=1 HUFF_DEC_VARIANT=$v timeout -k 10 120 python tools/kbench.py --phase decode --workload $w --iters 20)
  echo "w=$w v=$v $r"
done; done > gpurun_out/dec_sweep.log 2>&1
