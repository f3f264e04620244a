#!/usr/bin/env bash
# multi-kernel index-free decode: segment length sweep (HUFF_IDX_SEG)
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3h}; mkdir -p $out
cd $root
for w in zipf text; do for sg in 992 736 608 480 352; do
  HUFF_IDX_SEG=$sg timeout -k 10 120 python tools/kbench.py --phase indexless --workload $w --iters 10 > $out/idx_${w}_$sg.json 2>>$out/err.log || exit 1
done; done
for f in $out/idx_*.json; do echo "$(basename $f) $(python3 -c "import json;d=json.load(open('$f'));print(round(d['wall_ms_per_iter'],4))")"; done
