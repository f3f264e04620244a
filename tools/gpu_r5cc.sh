#!/usr/bin/env bash
# Round 5, pass cc: the staged segment record packed in one u64 (default) against lib/prev (HEAD: s, c, tm, dl in four arrays); earlier passes:
# exits written only where a fix-up reads them, against lib/prev (HEAD):
# index-free, fuzz, wide and file-path tests, alternated wall times, and the
# PMC profile of the index-free pipeline (traffic).
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5cc}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 600 python -u -m pytest tests/test_gpu_indexfree.py tests/test_gpu_parity.py tests/test_gpu_decode_check.py tests/test_gpu_fuzz.py tests/test_gpu_wide.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2 3; do
  for wl in zipf text; do
    for l in new prev; do
      if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
      timeout -k 10 200 python -u tools/kbench.py --phase indexless --workload $wl --iters 20 > $out/idx_${wl}_${l}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
    done
  done
done
unset HUFF_LIB_AB
for f in $out/idx_*.json; do echo "$(basename $f) $(grep -o '"wall_ms_per_iter": [0-9.]*' $f | tr '\n' ' ')"; done
bash tools/profile.sh indexless zipf ${tag}_idx_zipf > /dev/null 2>&1 || { echo "profile failed"; exit 1; }
echo done
