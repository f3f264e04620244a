#!/usr/bin/env bash
# ifd iteration: its tests, then index-free timing (single pass forced and
# gated vs the multi-kernel path) on Zipf and text.
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3d}; mkdir -p $out
cd $root
timeout -k 10 300 python -u -m pytest tests/test_gpu_ifd.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/ifd_tests.log 2>&1 || { tail -30 $out/ifd_tests.log; exit 1; }
tail -1 $out/ifd_tests.log
for w in zipf text; do for f in 2 0; do
  HUFF_IFD=$f timeout -k 10 120 python tools/kbench.py --phase indexless --workload $w --iters 10 > $out/idx_${w}_ifd${f}.json 2>>$out/err.log || exit 1
done; done
for f in $out/idx_*.json; do echo "$(basename $f) $(cat $f)"; done
