#!/usr/bin/env bash
# GPU suite, then the index-free paths: byte Zipf/text (kbench + kernel trace)
# and wide W = 2/4/8 (warm and cold)
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3z}; mkdir -p $out
cd $root
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for wl in zipf text; do
  timeout -k 10 120 python tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/${wl}_idx.json 2>>$out/err.log || exit 1
done
for w in 2 4 8; do
  timeout -k 10 180 python tools/wbench.py --width $w --iters 5 --indexless > $out/w${w}.json 2>>$out/err.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/idx_trace -o run --output-format csv -- python3 $root/tools/kbench.py --phase indexless --workload zipf --iters 5 > $out/idx_trace.log 2>&1 || { tail -5 $out/idx_trace.log; exit 1; }
cd $root
for f in $out/*.json; do echo "$(basename $f) $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d.get('indexless_decode_ms', d.get('wall_ms_per_iter')), d.get('indexless_decode_ms_cold',''))" $f)"; done
