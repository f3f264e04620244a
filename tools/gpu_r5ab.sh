#!/usr/bin/env bash
# Round 5, pass ab: the decode launch without an occupancy query on the
# one-shot grid (default) against lib/prev (HEAD: queried every launch):
# decode tests, alternated index-free walls and bench lines.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5ab}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 600 python -u -m pytest tests/test_gpu_indexfree.py tests/test_gpu_decode_check.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2 3; do
  for l in new prev; do
    if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
    timeout -k 10 200 python -u tools/kbench.py --phase indexless --workload zipf --iters 20 > $out/idx_zipf_${l}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
  done
done
unset HUFF_LIB_AB
for f in $out/idx_*.json; do echo "$(basename $f) $(grep -o '"wall_ms_per_iter": [0-9.]*' $f | tr '\n' ' ')"; done
echo done
