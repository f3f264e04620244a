#!/usr/bin/env bash
# Round 4: same-box A/B of variant libraries. Index-free decode (split path
# with a kernel trace, the older path, IDX_LIBS variants) and pass 1 (hist,
# HIST_LIBS variants), after a quick split-test pass.
#   IDX_LIBS="esum" HIST_LIBS="h512" WIDE_LIBS="ilp2" tools/gpu_r4e.sh <tag>
# (WIDE_LIBS: the wide GPU tests under each variant first, then wbench W = 2, 4)
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r4e}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/split_tests.log 2>&1
rc=$?; tail -2 $out/split_tests.log; [ $rc = 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
for wl in zipf text; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/idx_$wl -o run --output-format csv -- python3 $root/tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/idx_$wl.json 2> $out/idx_$wl.err || { echo "kbench $wl failed"; tail -5 $out/idx_$wl.err; exit 1; }
  grep phase $out/idx_$wl.json
  HUFF_SPLIT=0 timeout -k 10 240 python3 $root/tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/idx_old_$wl.json 2> $out/idx_old_$wl.err || { echo "old $wl failed"; exit 1; }
  echo -n "old: "; grep phase $out/idx_old_$wl.json
  for l in ${IDX_LIBS:-}; do
    HUFF_LIB_AB=$l timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/idx_${l}_$wl -o run --output-format csv -- python3 $root/tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/idx_${l}_$wl.json 2> $out/idx_${l}_$wl.err || { echo "$l $wl failed"; exit 1; }
    echo -n "$l: "; grep phase $out/idx_${l}_$wl.json
  done
done
cd $root
for rep in 1 2; do
  for wl in uniform zipf; do
    for l in new ${HIST_LIBS:-}; do
      if [ $l = new ]; then
        timeout -k 10 120 python tools/kbench.py --phase hist --workload $wl --iters 20 > $out/hist_${wl}_${l}_$rep.json 2>/dev/null || { echo "hist $l failed"; exit 1; }
      else
        HUFF_LIB_AB=$l timeout -k 10 120 python tools/kbench.py --phase hist --workload $wl --iters 20 > $out/hist_${wl}_${l}_$rep.json 2>/dev/null || { echo "hist $l failed"; exit 1; }
      fi
      echo -n "hist $wl $l $rep: "; cat $out/hist_${wl}_${l}_$rep.json
    done
  done
done
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
      echo -n "wbench w$w $l $rep: "; python3 -c "import json,sys; d=json.loads(open('$out/wbench_w${w}_${l}_$rep.json').read().strip().splitlines()[-1]); print({k: v for k, v in d.items() if 'decode' in k or 'dec' in k})"
    done
  done
done
echo "r4e done"
