#!/usr/bin/env bash
# Round 5, pass ee: pass 1 with the row sum publishing the weights itself
# (lib/hpub: the last workgroup by ticket, no k_hist_publish launch) against
# the default (k_rows_sum + k_hist_publish): GPU tests on lib/hpub, then
# alternated pass-1 times (kbench --phase hist, event-timed) and bench lines.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5ee}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 600 env HUFF_LIB_AB=hpub python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2 3; do
  for wl in uniform zipf; do
    for l in new hpub; do
      if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
      timeout -k 10 200 python -u tools/kbench.py --phase hist --workload $wl --iters 50 > $out/hist_${wl}_${l}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
    done
  done
done
for l in new hpub new hpub; do
  if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --file-path none --no-other-scaling --side none --no-general > $out/bench_$l.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$out/bench_$l.json').read().strip().splitlines()[-1]); print('$l', d['value'], d['kernels']['hist']['avg_ms'])"
done
unset HUFF_LIB_AB
for f in $out/hist_*.json; do echo "$(basename $f) $(grep -o '"hist_ms": [0-9.]*' $f)"; done
echo done
