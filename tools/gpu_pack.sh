#!/usr/bin/env bash
# pack-phase parity + timing (general kernels) on the three workloads
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pack_tests.log 2>&1
for w in zipf text uniform; do
  r=$(HUFF_DISABLE_FIXED8=1 timeout -k 10 120 python tools/kbench.py --phase pack --workload $w --iters 20); echo "w=$w $r"
done > gpurun_out/pack_sweep.log 2>&1
