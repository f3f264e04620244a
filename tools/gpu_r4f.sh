#!/usr/bin/env bash
# Round 4: PMC profiles of the split index-free decoder (default build and
# the LIBS variants) on Zipf, then the wide-decoder variants (WIDE_LIBS).
#   LIBS="ovl" WIDE_LIBS="ilp2" tools/gpu_r4f.sh <tag>
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r4f}
cd $root
bash tools/profile.sh indexless zipf ${tag}_idx_zipf > /dev/null 2>&1 || { echo "profile failed"; exit 1; }
echo "profile default done"
for l in ${LIBS:-}; do
  HUFF_LIB_AB=$l bash tools/profile.sh indexless zipf ${tag}_idx_${l}_zipf > /dev/null 2>&1 || { echo "profile $l failed"; exit 1; }
  echo "profile $l done"
done
out=$root/gpurun_out/$tag; mkdir -p $out
for l in ${WIDE_LIBS:-}; do
  HUFF_LIB_AB=$l timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/wide_tests_$l.log 2>&1
  rc=$?; echo -n "wide tests $l: "; tail -1 $out/wide_tests_$l.log; [ $rc = 0 ] || exit 1
done
for rep in 1 2; do
  for w in 2 4; do
    for l in new ${WIDE_LIBS:-}; do
      if [ $l = new ]; then
        timeout -k 10 180 python tools/wbench.py --width $w --iters 5 > $out/wbench_w${w}_${l}_$rep.json 2>/dev/null || { echo "wbench $l failed"; exit 1; }
      else
        HUFF_LIB_AB=$l timeout -k 10 180 python tools/wbench.py --width $w --iters 5 > $out/wbench_w${w}_${l}_$rep.json 2>/dev/null || { echo "wbench $l failed"; exit 1; }
      fi
      echo -n "wbench w$w $l $rep: "; python3 -c "import json; d=json.loads(open('$out/wbench_w${w}_${l}_$rep.json').read().strip().splitlines()[-1]); print({k: v for k, v in d.items() if 'dec' in k})"
    done
  done
done
echo "r4f done"
