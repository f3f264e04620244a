#!/usr/bin/env bash
# Round 6: the software-pipelined pack (HUFF_PACK_PIPE) - parity tests of the
# encode paths, then a same-box A/B against lib/ab (the unpipelined build,
# tools/build_variant.sh ab "-DHUFF_PACK_PIPE=0" csrc/device/pack.hip),
# kbench --phase pack on Zipf, text and uniform through the general kernels.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6pack}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_configs.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2 3; do
  for w in zipf text uniform; do
    for v in ab new; do
      lib=$([ $v = ab ] && echo ab || echo "")
      HUFF_DISABLE_FIXED8=1 HUFF_LIB_AB=$lib timeout -k 10 120 python tools/kbench.py --phase pack --workload $w --iters 20 > $out/${w}_${v}_$rep.json 2>/dev/null || { echo "kbench $w $v failed"; exit 1; }
      echo "$w $v $(python3 -c "import json;print(round(json.load(open('$out/${w}_${v}_$rep.json'))['pack_ms'],4))")"
    done
  done
done
