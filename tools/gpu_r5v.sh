#!/usr/bin/env bash
# Round 5, pass v (as u, the row halves for <= 2-byte letters only): the wide task decoder with 2 KiB transpose rows, buffer
# stores and up to 16 waves for <= 2-byte letters (default) against lib/w12
# (the same with the 12-wave cap) and lib/prev (HEAD): wide tests, then
# wbench W = 2, 4, 8 alternated.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5w}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 500 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_fuzz.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2; do
  for w in 2 4 8; do
    for l in new prev; do
      if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
      timeout -k 10 200 python -u tools/wbench.py --width $w --iters 10 > $out/wb_w${w}_${l}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
    done
  done
done
unset HUFF_LIB_AB
for f in $out/wb_*.json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print({k: v for k, v in d.items() if 'ms' in k})")"; done
