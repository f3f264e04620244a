#!/usr/bin/env bash
# Wide-letter timings at 1 GiB for widths 2, 4, 8 (+ index-free decode).
set -euo pipefail
out=gpurun_out/wbench
mkdir -p $out
for w in 2 4 8; do
  timeout -k 10 300 python tools/wbench.py --width $w --indexless > $out/w$w.json 2> $out/w$w.err
done
