#!/usr/bin/env bash
# Round 5, pass zz2: k_pack with 16 table copies (lib/c16: 16 KiB table, 4
# resident workgroups = 8 waves per SIMD, the persistent grid clamped to
# residency) against 32 copies (default: 3 workgroups, 6 waves per SIMD):
# parity tests on lib/c16, alternated kbench --phase pack.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5zz2}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 400 env HUFF_LIB_AB=c16 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rep in 1 2 3; do
  for wl in zipf text; do
    for l in new c16; do
      if [ $l = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$l; fi
      timeout -k 10 200 python -u tools/kbench.py --phase pack --workload $wl --iters 20 > $out/pack_${wl}_${l}_$rep.json 2> $out/err.log || { tail -20 $out/err.log; exit 1; }
    done
  done
done
unset HUFF_LIB_AB
for f in $out/pack_*.json; do echo "$(basename $f) $(grep -o '"pack_ms": [0-9.]*\|"pack": {[^}]*}' $f | head -1)"; done
echo done
