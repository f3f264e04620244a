#!/usr/bin/env bash
# Round 6: the index-free skip decoder's skip codes in one wave-uniform
# predicated loop (default) against the per-lane loop (lib/skipold, built
# with -DHUFF_SKIP_UNIFORM=0) and the exec-masked unrolled loop (lib/skipmask, =2): the GPU suite, then alternated same-box kbench
# runs of the index-free decode (verified) and a kernel trace of each.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-skipu}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2 3; do
  for w in zipf text; do
    for l in new skipold skipmask; do
      if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
      timeout -k 10 120 python tools/kbench.py --phase indexless --workload $w --iters 20 > $out/${w}_${l}_$rep.json 2>> $out/err.log || { tail -5 $out/err.log; exit 1; }
      echo "$w $l $rep $(python3 -c "import json; d=json.load(open('$out/${w}_${l}_$rep.json')); print(round(d['wall_ms_per_iter'],4))")"
    done
  done
done
unset HUFF_LIB_AB
cd /tmp && export TMPDIR=/tmp
for l in new skipold skipmask; do
  if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace_$l -o run --output-format csv -- python3 $root/tools/kbench.py --phase indexless --workload zipf --iters 10 > /dev/null 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('$out/trace_$l/run_kernel_stats.csv')):
    if 'spec_lds' in r['Name'] or 'fixed_skip' in r['Name']: print('$l', r['Name'][:40], r['AverageNs'])"
done
