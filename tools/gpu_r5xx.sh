#!/usr/bin/env bash
# Round 5, pass xx: index-free segments of 736 and 672 bits (lib/seg736, lib/seg672: 5 staged workgroups per CU) against 992 (4 per CU):
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5xx}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 600 env HUFF_LIB_AB=seg736 python -u -m pytest tests/test_gpu_indexfree.py tests/test_gpu_decode_check.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2 3; do
  for wl in zipf text; do
    for l in new seg736 seg672; do
      if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
      timeout -k 10 200 python -u tools/kbench.py --phase indexless --workload $wl --iters 20 > $out/idx_${wl}_${l}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
    done
  done
done
unset HUFF_LIB_AB
for f in $out/idx_*.json; do echo "$(basename $f) $(grep -o '"wall_ms_per_iter": [0-9.]*' $f | tr '\n' ' ')"; done
echo done
