#!/usr/bin/env bash
# 4-byte letters through u32 table entries: wide GPU tests, wbench W = 2/4/8
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3ae}; mkdir -p $out
cd $root
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 180 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for w in 2 4 8; do
  timeout -k 10 180 python tools/wbench.py --width $w --iters 5 --indexless > $out/w${w}.json 2>>$out/err.log || exit 1
done
for f in $out/*.json; do echo "$(basename $f) $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['kernels']['wdecode']['avg_ms'], d['kernels']['wdecode']['frac_of_8TBps'], d['indexless_decode_ms'], d['decode_GBps_input'])" $f)"; done
