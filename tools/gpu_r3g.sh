#!/usr/bin/env bash
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3g}; mkdir -p $out
cd $root
for w in zipf text; do
  HUFF_LIB_AB=ifdstats HUFF_IFD=2 HUFF_IFD_TRACE=1 timeout -k 10 120 python tools/kbench.py --phase indexless --workload $w --iters 2 > $out/stats_${w}.json 2> $out/stats_${w}.err || exit 1
done
grep -h "ifd" $out/stats_*.err | sort | uniq -c
