#!/usr/bin/env bash
# Round 5: the decoders with the next task's index prefetched by persistent
# waves (default) against the one-shot grid (lib/nopf), indexed decode and
# index-free decode, Zipf and text, alternated; decode tests first.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5f}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_indexfree.py tests/test_gpu_decode_check.py tests/test_gpu_fuzz.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2 3; do
  for wl in zipf text; do
    for v in new nopf; do
      if [ $v = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$v; fi
      timeout -k 10 200 python -u tools/kbench.py --phase decode --workload $wl --iters 20 > $out/dec_${wl}_${v}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
      timeout -k 10 200 python -u tools/kbench.py --phase indexless --workload $wl --iters 20 > $out/idx_${wl}_${v}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
      unset HUFF_LIB_AB
    done
  done
done
for f in $out/dec_*.json $out/idx_*.json; do echo "$(basename $f) $(grep -o '"decode_ms": [0-9.]*\|"wall_ms_per_iter": [0-9.]*' $f | tr '\n' ' ')"; done
