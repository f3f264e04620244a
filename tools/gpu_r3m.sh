#!/usr/bin/env bash
# (1) parity of the swizzled pack stage (in-tree), (2) pack A/B vs lib/noswz,
# (3) wide lane-bytes / prefetch A/B (lib/w16a1, w16a2, wmix)
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3m}; mkdir -p $out
cd $root
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py tests/test_gpu_configs.py -q -x -p no:cacheprovider --timeout 180 --timeout-method thread > $out/tests.log 2>&1; rc=$?
tail -3 $out/tests.log
[ $rc = 0 ] || { grep -E "FAILED|Error|assert" $out/tests.log | head -30; exit 1; }
for rep in 1 2; do
for v in base noswz; do
  for wl in zipf text; do
    if [ $v = base ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$v; fi
    timeout -k 10 120 python -u tools/kbench.py --phase pack --workload $wl --iters 20 > $out/kb_${v}_${wl}_$rep.json 2> $out/kb_${v}_${wl}_$rep.err || { tail -20 $out/kb_${v}_${wl}_$rep.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$out/kb_${v}_${wl}_$rep.json').read().strip().splitlines()[-1]);print('$v','$wl',$rep,round(d['pack_ms'],4))"
  done
done
done
for v in base w16a1 w16a2 wmix; do
  for w in 2 4; do
    if [ $v = base ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$v; fi
    timeout -k 10 200 python -u tools/wbench.py --width $w --iters 10 > $out/wb_${v}_w$w.json 2> $out/wb_${v}_w$w.err || { tail -20 $out/wb_${v}_w$w.err; exit 1; }
    python3 -c "import json;d=json.load(open('$out/wb_${v}_w$w.json'));k=d['kernels'];print('$v', $w, k['wbits']['avg_ms'], k['wpack']['avg_ms'], d['encode_GBps_input'])"
  done
done
