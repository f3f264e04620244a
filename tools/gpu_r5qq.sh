#!/usr/bin/env bash
# Round 5, pass qq: branch-free slow steps for trees whose slow windows are
# common (default) against the branching steps (HUFF_L2_SPARSE=1, same
# library): index-free and wide tests, alternated index-free walls.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5qq}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 600 python -u -m pytest tests/test_gpu_indexfree.py tests/test_gpu_wide.py tests/test_gpu_fuzz.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2; do
  for l in dense sparse; do
    if [ $l = dense ]; then unset HUFF_L2_SPARSE; else export HUFF_L2_SPARSE=1; fi
    for w in 2 4 8; do
      timeout -k 10 200 python -u tools/wbench.py --width $w --iters 5 --indexless > $out/w${w}_${l}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
    done
    for wl in zipf text; do
      timeout -k 10 200 python -u tools/kbench.py --phase indexless --workload $wl --iters 20 > $out/idx_${wl}_${l}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
    done
  done
done
unset HUFF_L2_SPARSE
for f in $out/idx_*.json; do echo "$(basename $f) $(grep -o '"wall_ms_per_iter": [0-9.]*' $f | tr '\n' ' ')"; done
for f in $out/w*.json; do echo "$(basename $f) $(grep -o '"indexless_decode_ms": [0-9.]*' $f | tr '\n' ' ')"; done
echo done
