#!/usr/bin/env bash
# Round 5, pass yy: the row sum over 2,048 and 4,096 workgroups (lib/rows2048, lib/rows4096) against 512 (default); kbench --phase hist, alternated.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5yy}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 300 env HUFF_LIB_AB=rows4096 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2 3; do
  for wl in uniform zipf; do
    for l in new rows2048 rows4096; do
      if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
      timeout -k 10 200 python -u tools/kbench.py --phase hist --workload $wl --iters 50 > $out/hist_${wl}_${l}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
    done
  done
done
unset HUFF_LIB_AB
for f in $out/hist_*.json; do echo "$(basename $f) $(grep -o '"hist_ms": [0-9.]*' $f)"; done
echo done
