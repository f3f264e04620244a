#!/usr/bin/env bash
# Round 5, pass ff: the wide task decoder's level-1 table width K1 = 10
# (default) against 11 and 12 bits (lib/k11, lib/k12; host-side table build
# only): wide GPU tests on both variants, alternated wbench W = 2 and 4.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5ff}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
for l in k11 k12; do
  timeout -k 10 400 env HUFF_LIB_AB=$l python -u -m pytest tests/test_gpu_wide.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests_$l.log 2>&1 || { tail -30 $out/gpu_tests_$l.log; exit 1; }
  tail -1 $out/gpu_tests_$l.log
done
for rep in 1 2 3; do
  for w in 2 4; do
    for l in new k11 k12; do
      if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
      timeout -k 10 200 python -u tools/wbench.py --width $w --iters 10 > $out/w${w}_${l}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
    done
  done
done
unset HUFF_LIB_AB
for f in $out/w*.json; do echo "$(basename $f) $(grep -o '"decode_ms": [0-9.]*' $f | tr '\n' ' ')"; done
echo done
