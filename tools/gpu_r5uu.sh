#!/usr/bin/env bash
# Round 5, pass uu: segments of ~640 and ~768 bits for trees with codes past the walk table (lib/seg640, lib/seg768: 4 staged workgroups per CU at 640) against the default 992:
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5uu}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 600 env HUFF_LIB_AB=seg640 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_indexfree.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2 3; do
  for l in new seg640 seg768; do
    if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
    for w in 2 4; do
      timeout -k 10 200 python -u tools/wbench.py --width $w --iters 5 --indexless > $out/w${w}_${l}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
    done
  done
done
unset HUFF_LIB_AB
for f in $out/w*.json; do echo "$(basename $f) $(grep -o '"indexless_decode_ms": [0-9.]*' $f | tr '\n' ' ')"; done
echo done
