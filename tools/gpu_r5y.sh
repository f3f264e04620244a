#!/usr/bin/env bash
# Round 5, pass y: k_pack issuing round r+1's table lookups right after round
# r's ORs (default) against lib/pe0 (lookups at the top of each round):
# parity tests, then kbench pack alternated (Zipf, text) and the bench's
# Zipf step.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5y}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py tests/test_gpu_mgpu.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2 3; do
  for wl in zipf text; do
    for l in new ${LIBS:-pe0}; do
      if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
      timeout -k 10 200 python -u tools/kbench.py --phase pack --workload $wl --iters 20 > $out/pack_${wl}_${l}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
    done
  done
done
unset HUFF_LIB_AB
for f in $out/pack_*.json; do echo "$(basename $f) $(grep -o '"pack_ms": [0-9.]*\|"pack": {[^}]*}' $f | head -2 | tr '\n' ' ')"; done
LIBS="${LIBS:-pe0}" REPS=2 BENCH_ARGS="--workload zipf" tools/gpu_benchab.sh $tag/benchab
