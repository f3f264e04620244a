#!/usr/bin/env bash
# Same-box A/B: decode (lib/ab = round-2 prologue) and index-free decode
# (single pass vs HUFF_IFD=0 multi-kernel), interleaved, 2 reps.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3c}; mkdir -p $out
cd $root
for rep in 1 2; do for w in zipf text; do
  for v in new ab; do
    if [ $v = new ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=ab; fi
    timeout -k 10 120 python tools/kbench.py --phase decode --workload $w --iters 20 > $out/dec_${w}_${v}_$rep.json 2>>$out/err.log || exit 1
  done
  unset HUFF_LIB_AB
  for f in 1 0; do
    HUFF_IFD=$f timeout -k 10 120 python tools/kbench.py --phase indexless --workload $w --iters 10 > $out/idx_${w}_ifd${f}_$rep.json 2>>$out/err.log || exit 1
  done
done; done
echo "r3c done"
