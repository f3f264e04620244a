#!/usr/bin/env bash
# Round 6: the speculative walk refilling every 4th / 3rd window for tables
# of <= 8 / <= 10 bits (default) against every 2nd (lib/walkr0,
# -DHUFF_WALK_R=0): the index-free, parity and wide tests, then alternated
# kbench index-free decodes of 1 GiB text and uniform through the general
# kernels (profiles/r06/walkr/).
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/walkr; mkdir -p $out
cd $root
timeout -k 10 400 python -u -m pytest tests/test_gpu_indexfree.py tests/test_gpu_parity.py tests/test_gpu_wide.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2 3; do
  for w in text uniform; do
    for l in new walkr0; do
      if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
      if [ $w = uniform ]; then export HUFF_DISABLE_FIXED8=1; else unset HUFF_DISABLE_FIXED8; fi
      timeout -k 10 120 python tools/kbench.py --phase indexless --workload $w --iters 20 > $out/${w}_${l}_$rep.json 2>> $out/err.log || { tail -5 $out/err.log; exit 1; }
      echo "$w $l $rep $(python3 -c "import json; d=json.load(open('$out/${w}_${l}_$rep.json')); print(round(d['wall_ms_per_iter'],4))")"
    done
  done
done
echo done
