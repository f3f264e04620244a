#!/usr/bin/env bash
# wide encoder A/B: lane bytes and prefetch depth (lib/<variant>)
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3l}; mkdir -p $out
cd $root
for v in base w16a1 w16a2 wmix base; do
  for w in 2 4 8; do
    if [ $v = base ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$v; fi
    timeout -k 10 200 python -u tools/wbench.py --width $w --iters 10 > $out/wb_${v}_w$w.json 2> $out/wb_${v}_w$w.err || { tail -20 $out/wb_${v}_w$w.err; exit 1; }
    python3 -c "import json;d=json.load(open('$out/wb_${v}_w$w.json'));k=d['kernels'];print('$v', $w, k['wbits']['avg_ms'], k['wpack']['avg_ms'], d['encode_GBps_input'])"
  done
done
