#!/usr/bin/env bash
set -euo pipefail
mkdir -p gpurun_out
: > gpurun_out/dec_tests3.log
for v in 3 4 5 6; do
  HUFF_DEC_VARIANT=$v timeout -k 10 300 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "medium or long or stitching" >> gpurun_out/dec_tests3.log 2>&1
done
for w in zipf text; do for v in 1 0 3 4 5 6; do
  r=$(HUFF_DISABLE_FIXED8=1 HUFF_DEC_VARIANT=$v timeout -k 10 120 python tools/kbench.py --phase decode --workload $w --iters 20)
  echo "w=$w v=$v $r"
done; done > gpurun_out/dec_sweep3.log 2>&1
