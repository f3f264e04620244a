#!/usr/bin/env bash
# k_ifd phase timing: builds that stop after each phase (IFD_STOP=1..5) and
# the full kernel, Zipf and text, single pass forced.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3e}; mkdir -p $out
cd $root
export HUFF_IFD=2
for w in zipf text; do for v in ifd1 ifd2 ifd3 ifd4 ifd5 full; do
  if [ $v = full ]; then unset HUFF_LIB_AB; else export HUFF_LIB_AB=$v; fi
  timeout -k 10 120 python tools/kbench.py --phase indexless --workload $w --iters 10 --no-verify > $out/${w}_$v.json 2>>$out/err.log || exit 1
done; done
for f in $out/*.json; do echo "$(basename $f) $(python3 -c "import json;d=json.load(open('$f'));print(round(d.get('ifd_kernel_ms',-1),4))")"; done
