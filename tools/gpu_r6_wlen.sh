#!/usr/bin/env bash
# Round 6: the wide decoder's length chain (2-byte letters, codes <= 16 bits)
# against the two-level chain (HUFF_WIDE_LEN_CHAIN=0): the wide tests, then
# alternated same-box wbench runs (W = 2, 1 GiB Zipf(1.1) over 4,096 letters;
# each verifies its round trip), indexed and index-free.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-wlen}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_fuzz.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for c in 0 1; do
    HUFF_WIDE_LEN_CHAIN=$c timeout -k 10 200 python tools/wbench.py --width 2 --iters 10 --indexless > $out/w2_c${c}_$r.json 2>> $out/err.log || { tail -5 $out/err.log; exit 1; }
    echo "W=2 len_chain=$c: $(cat $out/w2_c${c}_$r.json)"
  done
done
