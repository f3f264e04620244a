#!/usr/bin/env bash
# index-free A/B: current lib, nohalf (no half samples), skip0 (timing only: no skip codes)
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3aa}; mkdir -p $out
cd $root
for rep in 1 2; do for wl in zipf text; do
  timeout -k 10 120 python tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/${wl}_new_$rep.json 2>>$out/err.log || exit 1
  HUFF_LIB_AB=nohalf timeout -k 10 120 python tools/kbench.py --phase indexless --workload $wl --iters 10 > $out/${wl}_nohalf_$rep.json 2>>$out/err.log || exit 1
  HUFF_LIB_AB=skip0 timeout -k 10 120 python tools/kbench.py --phase indexless --workload $wl --iters 10 --no-verify > $out/${wl}_skip0_$rep.json 2>>$out/err.log || exit 1
done; done
for f in $out/*.json; do echo "$(basename $f) $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(round(d['wall_ms_per_iter'],4))" $f)"; done
