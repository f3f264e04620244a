#!/usr/bin/env bash
# Round 5, pass gg: kernel trace of the wide index-free decode (W = 2 and 4)
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=${1:-r5gg}
out=$root/gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for w in 2 4; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/trace_w$w -o run --output-format csv -- python3 $root/tools/wbench.py --width $w --iters 5 --indexless > $out/wbench_w$w.json 2> $out/trace_w$w.log || { tail -20 $out/trace_w$w.log; exit 1; }
done
echo done
