#!/usr/bin/env bash
# Round 5, pass z: pass 1 with two bins per dword (16-bit counters, 16 KiB
# image; default) against lib/pair0 (32 KiB of u32 counters): pass-1 tests,
# kbench hist alternated (uniform, Zipf, text), then the bench step A/B.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5z}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_mgpu.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2 3; do
  for wl in uniform zipf text; do
    for l in new pair0; do
      if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
      timeout -k 10 200 python -u tools/kbench.py --phase hist --workload $wl --iters 20 > $out/hist_${wl}_${l}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
    done
  done
done
unset HUFF_LIB_AB
for f in $out/hist_*.json; do echo "$(basename $f) $(grep -o '"hist_ms": [0-9.]*' $f)"; done
LIBS=pair0 REPS=3 tools/gpu_benchab.sh $tag/benchab
