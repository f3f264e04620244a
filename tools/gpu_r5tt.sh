#!/usr/bin/env bash
# Round 5, pass tt: the wide-letter benches (decode and index-free) of the last build
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5tt}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
for w in 2 4 8; do
  timeout -k 10 180 python tools/wbench.py --width $w --iters 10 --indexless > $out/wbench_w$w.json 2>>$out/wbench.err || { echo "wbench $w failed"; exit 1; }
done
echo done
