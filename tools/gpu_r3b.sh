#!/usr/bin/env bash
# Round 3: the single-pass index-free decoder's tests, then the full GPU suite
# and smoke, then same-box decode A/B (lib/ab = round-2 prologue) and the
# index-free decode single-pass vs multi-kernel (HUFF_IFD=0).
set -uo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/${1:-r3b}; mkdir -p $out
cd $root
timeout -k 10 300 python -u -m pytest tests/test_gpu_ifd.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $out/ifd_tests.log 2>&1 || { tail -40 $out/ifd_tests.log; exit 1; }
tail -2 $out/ifd_tests.log
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -2 $out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
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
echo "r3b done"
