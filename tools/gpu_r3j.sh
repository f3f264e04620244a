#!/usr/bin/env bash
# wide-letter encoder rewrite: wide tests, then wbench u16/u32/u64
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3j}; mkdir -p $out
cd $root
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -q -x -p no:cacheprovider --timeout 180 --timeout-method thread > $out/wide_tests.log 2>&1; rc=$?
tail -3 $out/wide_tests.log
[ $rc = 0 ] || { grep -E "FAILED|Error|assert" $out/wide_tests.log | head -30; exit 1; }
for w in 2 4 8; do
  timeout -k 10 200 python -u tools/wbench.py --width $w --iters 10 > $out/wbench_w$w.json 2> $out/wbench_w$w.err || { tail -20 $out/wbench_w$w.err; exit 1; }
  cat $out/wbench_w$w.json
done
