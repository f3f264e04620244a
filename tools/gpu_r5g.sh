#!/usr/bin/env bash
# Round 5: the decoders' 3 KiB stage (8 workgroups per CU, unswizzled) for
# streams of <= 5.6 bits per symbol: decode tests, then indexed and
# index-free decode against HUFF_SMALL_STAGE=0 (4.5 KiB stage), alternated,
# and the stamps.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5g}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_indexfree.py tests/test_gpu_decode_check.py tests/test_gpu_fuzz.py tests/test_gpu_configs.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2 3; do
  for wl in zipf text; do
    for v in 1 0; do
      HUFF_SMALL_STAGE=$v timeout -k 10 200 python -u tools/kbench.py --phase decode --workload $wl --iters 20 > $out/dec_${wl}_s${v}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
      HUFF_SMALL_STAGE=$v timeout -k 10 200 python -u tools/kbench.py --phase indexless --workload $wl --iters 20 > $out/idx_${wl}_s${v}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
    done
  done
done
for f in $out/dec_*.json $out/idx_*.json; do echo "$(basename $f) $(grep -o '"decode_ms": [0-9.]*\|"wall_ms_per_iter": [0-9.]*' $f | tr '\n' ' ')"; done
HUFF_LIB_AB=stamps timeout -k 10 200 python -u tools/stamps.py --workload zipf > $out/stamps_zipf.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
