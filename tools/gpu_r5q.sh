#!/usr/bin/env bash
# Round 5, pass q: k_fix_list loads its table only when a seam differs, k_mark_lite reads the true start only when a mark needs it, against
# lib/prev (HEAD): index-free tests, alternated wall
# times, stamps of both, and a kernel trace of the default pipeline.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5q}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
HUFF_FIX_STATS=1 timeout -k 10 120 python -u -m pytest tests/test_gpu_indexfree.py -k "fix_chain or matches_oracle or lead_in" -s -q -p no:cacheprovider > $out/fix_stats.log 2>&1 || { tail -30 $out/fix_stats.log; exit 1; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_indexfree.py tests/test_gpu_parity.py tests/test_gpu_decode_check.py tests/test_gpu_fuzz.py tests/test_gpu_wide.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
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
HUFF_LIB_AB=stamps timeout -k 10 200 python -u tools/stamps.py --workload zipf > $out/stamps_zipf.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/idx_trace -o run --output-format csv -- python3 $root/tools/kbench.py --phase indexless --workload zipf --iters 5 > $out/idx_trace.log 2>&1 || { tail -20 $out/idx_trace.log; exit 1; }
echo done
