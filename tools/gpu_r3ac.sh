#!/usr/bin/env bash
# wide index-free decode with k_mark_lite + skip codes: wide GPU tests, then
# wbench W = 2/4/8 (skip marks vs walked marks, same box)
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3ac}; mkdir -p $out
cd $root
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 180 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for w in 2 4 8; do
  timeout -k 10 180 python tools/wbench.py --width $w --iters 5 --indexless > $out/w${w}_skip.json 2>>$out/err.log || exit 1
  HUFF_WIDE_MARK_WALK=1 timeout -k 10 180 python tools/wbench.py --width $w --iters 5 --indexless > $out/w${w}_walk.json 2>>$out/err.log || exit 1
done
for f in $out/*.json; do echo "$(basename $f) $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['indexless_decode_ms'], d['indexless_decode_ms_cold'], d['kernels']['wdecode']['avg_ms'])" $f)"; done
