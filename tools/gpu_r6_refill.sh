#!/usr/bin/env bash
# Round 6: lookups per window refill in the fixed-count decoders (R = 4 for
# trees of <= 8 bits, 3 for <= 10) against two (HUFF_DEC_REFILL=2): the GPU
# suite, then alternated same-box kbench runs of the general decode and the
# index-free decode on 1 GiB uniform through the general kernels
# (HUFF_DISABLE_FIXED8=1), and a kernel trace of each (profiles/r06/refill/).
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/refill; mkdir -p $out
cd $root
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
export HUFF_DISABLE_FIXED8=1
for rep in 1 2 3; do
  for ph in decode indexless; do
    for r in auto 2; do
      if [ $r = auto ]; then unset HUFF_DEC_REFILL; else export HUFF_DEC_REFILL=$r; fi
      timeout -k 10 120 python tools/kbench.py --phase $ph --workload uniform --iters 20 > $out/${ph}_r${r}_$rep.json 2>> $out/err.log || { tail -5 $out/err.log; exit 1; }
      echo "$ph $r $rep $(python3 -c "import json; d=json.load(open('$out/${ph}_r${r}_$rep.json')); print({k: v for k, v in d.items() if 'ms' in k})")"
    done
  done
done
unset HUFF_DEC_REFILL
cd /tmp && export TMPDIR=/tmp
for r in auto 2; do
  if [ $r = auto ]; then unset HUFF_DEC_REFILL; else export HUFF_DEC_REFILL=$r; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace_$r -o run --output-format csv -- python3 $root/tools/kbench.py --phase decode --workload uniform --iters 10 > /dev/null 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('$out/trace_$r/run_kernel_stats.csv')):
    if 'decode_fixed' in r['Name']: print('$r', r['Name'][:60], r['AverageNs'])"
done
echo done
