#!/usr/bin/env bash
# Round 6: a pack variant library (V=acc: the accumulator emit,
# emit_codes_acc; V=c16: 16 table copies, more workgroups per CU) against the
# default: parity under the variant, then kbench
# --phase pack on Zipf, text and uniform through the general kernels, and the
# Zipf bench line, alternated.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r6acc}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
HUFF_LIB_AB=${V:-acc} timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1; tail -2 $out/pytest.log
V=${V:-acc}
for r in 1 2; do
  for v in default $V; do
    if [ $v = default ]; then env=""; else env="HUFF_LIB_AB=$v"; fi
    for wl in zipf text uniform; do
      fx=""; [ $wl = uniform ] && fx="HUFF_DISABLE_FIXED8=1"
      env $env $fx timeout -k 10 120 python -u tools/kbench.py --phase pack --workload $wl --iters 20 > $out/pack_${v}_${wl}_$r.json 2> $out/pack_${v}_${wl}_$r.err || { tail -5 $out/pack_${v}_${wl}_$r.err; exit 1; }
    done
  done
done
grep -H "pack" $out/pack_*.json | sed "s|$out/||" | cut -c1-200
