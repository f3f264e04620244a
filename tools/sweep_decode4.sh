#!/usr/bin/env bash
set -euo pipefail
mkdir -p gpurun_out
HUFF_DEC_VARIANT=7 timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/dec_tests4.log 2>&1
for w in zipf text uniform; do for v in 3 7; do
  r=$(HUFF_DISABLE_FIXED8=1 HUFF_DEC_VARIANT=$v timeout -k 10 120 python tools/kbench.py --phase decode --workload $w --iters 20)
  echo "w=$w v=$v $r"
done; done > gpurun_out/dec_sweep4.log 2>&1
