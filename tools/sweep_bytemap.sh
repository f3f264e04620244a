#!/usr/bin/env bash
# byte-map kernel variant x grid sweep (pack phase, 1 GiB uniform)
set -e; mkdir -p gpurun_out
for v in 0 1 2 3 4; do for g in 1024 2048 4096 100000; do
  r=$(HUFF_BM_VARIANT=$v HUFF_BM_GRID=$g timeout -k 10 120 python tools/kbench.py --phase pack --workload uniform --iters 20)
  echo "v=$v g=$g $r"
done; done > gpurun_out/bm_sweep.log 2>&1
