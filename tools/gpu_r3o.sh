#!/usr/bin/env bash
# wide task decoder (wdecode.hip) + 64-letter restart index: tests, wbench; batch trees after the load fix
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3o}; mkdir -p $out
cd $root
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_batch.py -q -x -p no:cacheprovider --timeout 180 --timeout-method thread > $out/tests.log 2>&1; rc=$?
tail -3 $out/tests.log
[ $rc = 0 ] || { grep -E "FAILED|Error|assert" $out/tests.log | head -30; exit 1; }
for w in 2 4 8; do
  timeout -k 10 200 python -u tools/wbench.py --width $w --iters 10 --indexless > $out/wbench_w$w.json 2> $out/wbench_w$w.err || { tail -20 $out/wbench_w$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/wbench_w$w.json'));k=d['kernels'];print($w, 'bits',k['wbits']['avg_ms'], 'pack',k['wpack']['avg_ms'], 'dec',k['wdecode']['avg_ms'], k['wdecode']['frac_of_8TBps'], 'enc',d['encode_GBps_input'], 'dec',d['decode_GBps_input'], 'idxfree', d.get('indexless_decode_ms'))"
done
timeout -k 10 200 python -u tools/batchbench.py --streams 10000 --bytes 16384 > $out/batch.json 2> $out/batch.err || { tail -20 $out/batch.err; exit 1; }
cat $out/batch.json
