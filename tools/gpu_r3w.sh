#!/usr/bin/env bash
# k_ifd phase timestamps (IFD_DBG variant build lib/dbg) on 1 GiB Zipf and text
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3w}; mkdir -p $out
cd $root
for w in zipf text; do
  HUFF_LIB_AB=dbg HUFF_IFD=2 HUFF_IFD_DBG=$out/${w}_dbg.bin timeout -k 10 120 python tools/kbench.py --phase indexless --workload $w --iters 3 > $out/${w}_dbg.json 2>$out/${w}_dbg.err || exit 1
done
ls -la $out
