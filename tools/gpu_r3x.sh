#!/usr/bin/env bash
# level-2 length table for the sync kernels: wide + parity GPU tests, then the
# wide index-free decode with and without it (HUFF_NO_L2=1), and the byte
# index-free path on Zipf/text (same box)
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3x}; mkdir -p $out
cd $root
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for w in 2 4 8; do
  timeout -k 10 180 python tools/wbench.py --width $w --iters 5 --indexless > $out/w${w}_l2.json 2>>$out/err.log || exit 1
  HUFF_NO_L2=1 timeout -k 10 180 python tools/wbench.py --width $w --iters 5 --indexless > $out/w${w}_nol2.json 2>>$out/err.log || exit 1
done
for wl in zipf text; do
  timeout -k 10 120 python tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/${wl}_l2.json 2>>$out/err.log || exit 1
  HUFF_NO_L2=1 timeout -k 10 120 python tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/${wl}_nol2.json 2>>$out/err.log || exit 1
done
for f in $out/*.json; do echo "$(basename $f) $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d.get('indexless_decode_ms', d.get('wall_ms_per_iter')))" $f)"; done
