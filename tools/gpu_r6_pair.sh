#!/usr/bin/env bash
# Round 6: the two-chain wide decoder (k_wdec_pair) — its GPU tests, then
# wbench with HUFF_WIDE_PAIR=0 (one-task decoder) and =1 alternated on one box
# (profiles/r06/wide_pair/)
set -euo pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/pair
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
for i in 1 2; do
  for m in 0 1; do
    HUFF_WIDE_PAIR=$m timeout -k 10 150 python tools/wbench.py --width 2 --iters 10 --indexless > $O/w2_p${m}_$i.json
    tail -c 400 $O/w2_p${m}_$i.json
  done
done
for m in 0 1; do
  HUFF_WIDE_PAIR=$m timeout -k 10 150 python tools/wbench.py --width 4 --iters 10 --indexless > $O/w4_p${m}.json
done
echo done
