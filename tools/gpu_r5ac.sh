#!/usr/bin/env bash
# Round 5, pass ac: the indexed decoder in 16-wave workgroups sharing one
# table copy (lib/wg16: 8 waves per SIMD) against 4-wave workgroups (default:
# 6 per SIMD, LDS-bound): parity tests on lib/wg16, alternated kbench decode.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5ac}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 400 env HUFF_LIB_AB=wg16 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2 3; do
  for wl in zipf text; do
    for l in new wg16; do
      if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
      timeout -k 10 200 python -u tools/kbench.py --phase decode --workload $wl --iters 20 > $out/dec_${wl}_${l}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
    done
  done
done
unset HUFF_LIB_AB
for f in $out/dec_*.json; do echo "$(basename $f) $(grep -o '"decode_ms": [0-9.]*' $f | head -1)"; done
echo done
