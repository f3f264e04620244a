#!/usr/bin/env bash
# Round 6: codes per window refill in the wide task decoder (RF = 4 for
# codes of <= 8 bits, 3 for <= 10) against two (HUFF_DEC_REFILL=2): the wide
# and byte parity suites, then alternated wbench runs of u16 letters over 32
# and 100 letters (profiles/r06/wrefill/).
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/wrefill; mkdir -p $out
cd $root
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
  for k in 32 100; do
    for r in auto 2; do
      if [ $r = auto ]; then unset HUFF_DEC_REFILL; else export HUFF_DEC_REFILL=$r; fi
      timeout -k 10 150 python tools/wbench.py --width 2 --alphabet $k --iters 10 --indexless > $out/w2_k${k}_r${r}_$rep.json 2>> $out/err.log || { tail -5 $out/err.log; exit 1; }
      echo "k=$k r=$r $rep $(python3 -c "import json; d=json.loads(open('$out/w2_k${k}_r${r}_$rep.json').read().strip().splitlines()[-1]); print(d['bits_per_letter'], d['kernels']['wdecode']['avg_ms'], d['indexless_decode_ms'])")"
    done
  done
done
echo done
