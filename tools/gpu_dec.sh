#!/usr/bin/env bash
# Decode A/B: byte-path parity tests, then kbench decode timings per decode
# kernel (HUFF_DEC_VARIANT: 9 wave, 7 ring, 1 single-symbol) and workload.
#   tools/gpu_dec.sh [tag] [skip-tests]
set -euo pipefail
out=gpurun_out/${1:-dec}
mkdir -p $out
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1
fi
for w in zipf text; do
  for v in 10 9 7; do
    HUFF_DEC_VARIANT=$v timeout -k 10 200 python tools/kbench.py --phase decode --workload $w --iters 20 > $out/dec_${w}_$v.json 2> $out/dec_${w}_$v.err
  done
done
for v in 10 9 1; do
  HUFF_DISABLE_FIXED8=1 HUFF_DEC_VARIANT=$v timeout -k 10 200 python tools/kbench.py --phase decode --workload uniform --iters 20 > $out/dec_uniform_$v.json 2> $out/dec_uniform_$v.err
done
cat $out/dec_*.json
