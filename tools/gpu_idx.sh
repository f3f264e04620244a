#!/usr/bin/env bash
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "dev_decompress or foreign or compress_matches" > gpurun_out/idx_tests.log 2>&1
for w in zipf text uniform; do
  timeout -k 10 200 python tools/kbench.py --phase indexless --workload $w --iters 5
done > gpurun_out/idx_sweep.log 2>&1
