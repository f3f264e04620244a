#!/usr/bin/env bash
# index-free segment size vs LDS occupancy: 992 bits (42.1 KB per workgroup:
# 3 per CU) against 928 / 864 (<= 40 KB: 4 per CU), same box, two reps
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3af}; mkdir -p $out
cd $root
for rep in 1 2; do for wl in zipf text; do for sg in 992 928 864; do
  HUFF_IDX_SEG=$sg timeout -k 10 120 python tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/${wl}_${sg}_$rep.json 2>>$out/err.log || exit 1
done; done; done
for f in $out/*.json; do echo "$(basename $f) $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(round(d['wall_ms_per_iter'],4))" $f)"; done
