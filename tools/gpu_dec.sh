#!/usr/bin/env bash
# Decode A/B: parity, then kbench decode timings for the ring decoder with
# 256- and 1024-lane workgroups (HUFF_RING_NT).
set -euo pipefail
out=gpurun_out/dec
mkdir -p $out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider > $out/tests.log 2>&1
for w in zipf text; do
  for nt in 256 1024; do
    HUFF_RING_NT=$nt timeout -k 10 200 python tools/kbench.py --phase decode --workload $w --iters 20 > $out/dec_${w}_$nt.json 2> $out/dec_${w}_$nt.err
  done
done
